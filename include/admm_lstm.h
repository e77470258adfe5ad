/*
 * admm_lstm.h -- C ABI of libadmmlstm.so, the MI355X (gfx950) implementation of the
 * ADMM-LSTM update step of Frederick2309/ADMM-LSTM.
 *
 * The reference has no FFI of its own: its hot path is the Python method
 * ADMMBasedOptimizer.step() (admm.py:62-78; variant admm.no_dual_y.py:52-66) and
 * the model-side forward LSTM.init_gate_variables / LSTM.forward
 * (blocks/lstm.py:43-46, 65-88).  Each entry point below replaces one of those
 * Python calls; the Python drop-in (admm-lstm_amd/admm.py) binds them with ctypes
 * exactly as shown in INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only: device pointers (float*), sizes, a hipStream_t passed as void*.
 *  - Every function returns 0 on success and a negative ADMM_E* code on failure;
 *    admm_last_error() returns the thread-local message of the last failure.
 *  - Enqueue-only: admm_step / admm_init_state / admm_forward never synchronise the
 *    host with the device; results are stream-ordered on the given stream.
 *  - Buffers are BORROWED: the caller (PyTorch) owns them, keeps them alive and
 *    contiguous, and re-binds (admm_bind) whenever a pointer changes.
 *  - Layouts are the reference's: x [B,T,D], y [B,O], gates/duals [B,T+1,H]
 *    (time index 0 = the zero initial state), weights x2q [D,H], h2q [H,H], out [H,O].
 *  - One context per (process, device).  Calls on one context are not thread-safe.
 */
#ifndef ADMM_LSTM_H
#define ADMM_LSTM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADMM_LSTM_ABI_VERSION 3

enum {
  ADMM_OK = 0,
  ADMM_EINVAL = -1,   /* bad argument / shape / parameter */
  ADMM_EHIP = -2,     /* HIP runtime error */
  ADMM_ENOMEM = -3,   /* device allocation failed */
  ADMM_ECOMM = -4,    /* RCCL error */
  ADMM_ESTATE = -5,   /* call not valid in the context's state (e.g. step before bind) */
  ADMM_EFAULT = -6    /* a step's device work failed an internal check (the column-split sweep's
                         hand-off timed out): the bound state is invalid until the caller rewrites
                         it (admm_init_state, or a restore followed by admm_ack_fault) */
};

enum { ADMM_VARIANT_ADMM = 0, ADMM_VARIANT_NO_DUAL_Y = 1 };

/* Gate order everywhere: i, f, g, o, c, h (admm.py:170; blocks/lstm.py:86-88). */
enum { ADMM_I = 0, ADMM_F = 1, ADMM_G = 2, ADMM_O = 3, ADMM_C = 4, ADMM_H = 5 };

typedef struct AdmmDims {
  int64_t batch;          /* rows held by this rank (train_x.size(0) of the shard) */
  int64_t global_batch;   /* rows over all ranks: the B of the a-update, admm.py:496-502 */
  int32_t seq_len;        /* T */
  int32_t input_size;     /* D */
  int32_t hidden_size;    /* H */
  int32_t output_size;    /* O */
} AdmmDims;

typedef struct AdmmParams {
  /* rho i,f,g,o,c,h,y   (parameters.py 'rho'; admm.py:148-162) */
  float rho[7];
  /* beta for x2i,x2f,x2g,x2o ('wi','wf','wg','wo') and h2i..h2o ('vi'..'vo'), and wy
     (parameters.py 'beta'; admm.py:126-146) */
  float beta_x[4];
  float beta_h[4];
  float beta_y;
  int32_t variant;        /* ADMM_VARIANT_ADMM (admm.py) or ADMM_VARIANT_NO_DUAL_Y (admm.no_dual_y.py) */
  int32_t with_dual_y;    /* module flag admm.with_dual_y (admm.py:12); admm variant only */
} AdmmParams;

typedef struct AdmmBuffers {
  const float* x;         /* [B,T,D] train_x shard */
  const float* y;         /* [B,O]   train_y shard */
  float* wx[4];           /* model.x2i .. x2o  [D,H] */
  float* wh[4];           /* model.h2i .. h2o  [H,H] */
  float* wy;              /* model.out [H,O] */
  float* gates[6];        /* optimizer.gates['i'..'h'] [B,T+1,H] */
  float* duals[6];        /* optimizer.duals['i'..'h'] [B,T+1,H] */
  float* a;               /* optimizer.gates['a'] [B,O] */
  float* dual_y;          /* optimizer.duals['y'] [B,O] */
} AdmmBuffers;

/* Per-step diagnostics (admm_get_stats; the only call that synchronises). */
typedef struct AdmmStats {
  int32_t steps;              /* steps run on this context */
  int32_t k[8];               /* chosen line-search exponent of the last step, order
                                 (x,i),(h,i),(x,f),(h,f),(x,g),(h,g),(x,o),(h,o) (admm.py:69-71):
                                 theta* = 2^k / 2 (admm.py:331-338) */
  int32_t passes[2];          /* trial passes used by the x and h stage searches */
  double f_w[8];              /* objective f(W) of each weight search (admm.py:316-325) */
  double grad_sq[8];          /* ||G||^2 of each weight search */
  float theta_h;              /* theta* of the h_T search (admm.py:474-482) */
  int32_t unresolved;         /* weight searches that hit the candidate cap (should be 0) */
  int32_t nonfinite;          /* NaN/Inf seen in line-search sums (should be 0) */
  double direct_frac[8];      /* fraction of elements outside the polynomial regime of each
                                 weight search (|q| > 2^-5: per-candidate evaluation) */
  /* ABI 2 */
  int32_t handoff_fail;       /* column-split sweep hand-off waits that timed out, running count
                                 (any growth invalidates the state: admm_step then fails ADMM_EFAULT) */
  int32_t sweep_fallbacks;    /* column-split sweep launches whose grid was not all resident at once,
                                 running count: the row-block sweep did that step's sweep (slower) */
  int32_t graph_captures;     /* ADMM_GRAPH=1: step graphs captured */
  int32_t graph_disabled;     /* 1 once a capture failed: steps run eagerly from then on */
  int64_t graph_replays;      /* steps run as a replay of a captured graph */
  int32_t sweep_split_off;    /* 1 once 3 column-split launches fell back: the context then runs the
                                 row-block sweep directly (no entry wait per step) */
} AdmmStats;

typedef struct AdmmCtx AdmmCtx;

/* ABI version (ADMM_LSTM_ABI_VERSION) and the gfx arch the library was built for. */
int32_t admm_abi_version(void);
const char* admm_build_info(void);
const char* admm_last_error(void);

/* ADMMBasedOptimizer.__init__ (admm.py:34-60): validates dims/params, allocates the
   device workspace (z cache, residual/trial scratch, packed weights). */
int admm_create(const AdmmDims* dims, const AdmmParams* params, int device, AdmmCtx** out);
int admm_destroy(AdmmCtx* ctx);

/* Point the context at the caller-owned tensors (admm.py:45-60 attributes). Invalidates
   the z cache. */
int admm_bind(AdmmCtx* ctx, const AdmmBuffers* bufs);

/* Replaces admm.py:164-173 (__initialize_primal_gates / __initialize_dual_variables):
   gates <- LSTM forward of x (blocks/lstm.py:65-88), a <- h_T @ out, duals <- 0. */
int admm_init_state(AdmmCtx* ctx, void* stream);

/* Replaces ADMMBasedOptimizer.step() (admm.py:62-78 / admm.no_dual_y.py:52-66). */
int admm_step(AdmmCtx* ctx, void* stream);

/* The module flag admm.with_dual_y is read at every step in the reference (admm.py:77,
   255, 461, 498); the drop-in forwards its current value before each admm_step. */
int admm_set_with_dual_y(AdmmCtx* ctx, int32_t flag);

/* The library keeps caches derived from the bound state between steps: the z cache
   (x_t Wx + h_{t-1} Wh for every t, produced by the time sweep), the next x stage's targets
   tgt = dual/rho + gate and its X^T R partials (also left by the sweep), and the flag that the
   h dual is zero before T (which lets the sweep skip loading it).  Call this after ANY write
   outside admm_step to the weights, x, a gate plane or a dual plane (in particular the h dual
   at t < T, which would otherwise be read as zero); the next step then rebuilds them. */
int admm_invalidate_cache(AdmmCtx* ctx);

/* ABI 3.  Acknowledge the hand-off faults counted so far (AdmmStats::handoff_fail) after the
   caller has restored the bound state (e.g. from a checkpoint): admm_step stops failing with
   ADMM_EFAULT and the caches are invalidated as by admm_invalidate_cache.  Nothing else clears a
   fault except admm_init_state (re-binding and cache invalidation do not): an in-place edit of
   the invalid state is not a restore.  Replaces no reference interface (device faults have no
   reference analogue). */
int admm_ack_fault(AdmmCtx* ctx);

/* Multi-GPU (one process per GPU): rank 0 calls admm_comm_unique_id, the bytes are
   broadcast out of band (torch.distributed), every rank calls admm_set_comm.  All batch
   sums of the step are then all-reduced with RCCL over xGMI. */
int admm_comm_unique_id(void* out, int64_t out_bytes);
int admm_set_comm(AdmmCtx* ctx, const void* unique_id, int64_t id_bytes, int rank, int world);

/* Host-staged communicator, for hosts without RCCL and for testing the sharded step with
   several processes on one GPU (torch.distributed gloo): every all-reduce of admm_step
   synchronises the stream, copies the buffer to host memory and calls fn, which must sum
   `count` elements (dtype 0 = float32, 1 = float64) over all ranks in place and return 0.
   Replaces any RCCL communicator.  Not the performance path: each call is a host round trip. */
typedef int (*admm_host_allreduce_fn)(void* host_buf, int64_t count, int32_t dtype, void* user);
int admm_set_comm_host(AdmmCtx* ctx, admm_host_allreduce_fn fn, void* user, int rank, int world);

/* Synchronous: the diagnostics of the last step (line-search exponents etc.). */
int admm_get_stats(AdmmCtx* ctx, AdmmStats* out);

/* Non-blocking: the running counts of line searches that found no exponent in the
   searched window (admm.py:334-336 would keep doubling) and of
   non-finite objective values, as of the last step whose final kernel has completed
   (a host-mapped mirror; no device sync).  The drop-in warns when they grow. */
int admm_poll_status(AdmmCtx* ctx, int32_t* unresolved, int32_t* nonfinite);
/* ABI 2.  admm_poll_status also returns ADMM_EFAULT (with both counts filled) once a hand-off
   timeout is known.  admm_poll_faults: the running counts of AdmmStats::handoff_fail and
   ::sweep_fallbacks as of the last completed step (non-blocking, the same mirror). */
int admm_poll_faults(AdmmCtx* ctx, int32_t* handoff_fail, int32_t* sweep_fallbacks);

/* Live kernel timing (used by bench.py's roofline): when a class bit is set, admm_step
   records a hipEvent pair around every launch of that class on the step's stream.
   admm_profile_read waits for them, returns total ms and launch counts per class, and
   resets.  Classes: */
enum {
  ADMM_PROF_SWEEP = 0,        /* the time sweep: one persistent k_sweep_rows launch (or k_sweep_t per t) */
  ADMM_PROF_TRIAL = 1,        /* first line-search trial pass of the x stage */
  ADMM_PROF_TRIAL_EXTRA = 2,  /* the tail trial pass, windows 1..3 (exits at once when every gate is resolved) */
  ADMM_PROF_ATR_X = 3,        /* G = X^T R (x stage) */
  ADMM_PROF_ATR_H = 4,        /* G = Hprev^T R (h stage) */
  ADMM_PROF_QGEMM_X = 5,      /* Q = X G */
  ADMM_PROF_QGEMM_H = 6,      /* Q = Hprev G */
  ADMM_PROF_RESID = 7,        /* residual / target pass of each weight stage */
  ADMM_PROF_SMALL = 8,        /* wy and h_T kernels */
  ADMM_PROF_ZGEMM = 9,        /* z-cache recompute (only after external modifications) */
  ADMM_PROF_COMM = 10,        /* RCCL all-reduces */
  ADMM_PROF_TRIAL_H = 11,     /* first line-search trial pass of the h stage */
  ADMM_PROF_CLASSES = 12
};
int admm_profile(AdmmCtx* ctx, uint32_t class_mask);
int admm_profile_read(AdmmCtx* ctx, double* ms /* [ADMM_PROF_CLASSES] */, int32_t* count /* [ADMM_PROF_CLASSES] */);

/* Test hook (synchronous): the line-search trial arithmetic of one gate on caller data.
   out[k] (host, 16 doubles) = sum_e [(phi(z_e + q_e 2^-(kbase+k)) - tgt_e)^2 - (phi(z_e) - tgt_e)^2],
   phi = tanh if (tanh_gate & 1) else sigmoid (the increment form of admm.py:316-334).
   tanh_gate & 2: with the fast kernels' packed pair arithmetic instead of the generic kernels'
   per-element one. */
int admm_debug_trial(const float* z, const float* tgt, const float* q, int64_t n, int32_t tanh_gate, int32_t kbase,
                     double* out, void* stream);

/* Test hook (synchronous): copy a workspace array of the context to device memory dst.
   which: 0 = z cache [4][B*T][H], 1 = targets lam/rho + S [4][B*T][H] (valid flag in the
   return value's sign: 1 if the next x stage will read it, 0 if it will recompute it),
   2 = the last h-side trial direction Q = Hprev G_h as stored (layout per ADMM_QPAIR; the
   first 4*B*T*H*4 bytes of its buffer, returns 1). */
int admm_debug_workspace(AdmmCtx* ctx, int32_t which, void* dst, int64_t bytes, void* stream);

/* Test hook: while set, every admm_step copies each weight stage's gradient G_q (rho-scaled,
   after the all-reduce: the search direction of admm.py:302-312) on the step's stream into the
   caller's device buffers: gx [4][D][H] (x stage), gh [4][H][H] (h stage).  NULL pointers
   turn the copy off.  The parity tests use it to arbitrate line-search exponents from the
   library's own search direction. */
int admm_debug_trace(AdmmCtx* ctx, float* gx, float* gh);

/* Test hook: while set, every admm_step also writes the residual each weight stage formed its
   gradient from, R_q = (phi(z) - dual/rho - gate) phi'(z) (admm.py:302-312), element by element as
   the stage's gradient kernel formed it (same activation code), into the caller's device buffers
   rx (x stage) and rh (h stage), each [4][B*T][H] with row b*T + (t-1).  With admm_debug_trace's
   G, a test recomputes G = rho A^T R on the identical operands (A = X or H_prev) in fp64 and
   measures the gradient GEMM's own arithmetic error.  NULL pointers turn the copy off. */
int admm_debug_trace_resid(AdmmCtx* ctx, float* rx, float* rh);

/* Test hook: replay given line-search decisions.  While set (k8 != NULL), every admm_step still
   runs each search but then applies k8[2 q + side] (q = i,f,g,o; side 0 = x2q, 1 = h2q) as the
   exponent of admm.py:331-343 and, for the h_T search (admm.py:474-482), theta = 0.1 doubled
   ht_fails times, halved.  The decisions the step would have taken itself are read back with
   admm_debug_own (k = -1: not decided within the first window of 16 exponents).  The parity
   tests use it to follow a reference trajectory whose fp32 decisions are rounding noise
   (C1 on GoogleStock) and to arbitrate the step's own decisions along it.  k8 == NULL: off. */
int admm_debug_force(AdmmCtx* ctx, const int32_t* k8, int32_t ht_fails);
/* Test hook (ABI 2): one-shot fault injection into the next admm_step.  kind 1: in the column-split
   sweep, row block 0's column group 1 skips its publish of h_1, so the other groups' hand-off waits
   time out (ADMM_ESTATE if the context has no column split); kind 2: the next step-graph capture
   (ADMM_GRAPH=1) fails as if hipGraphInstantiate had; 0: clear. */
int admm_debug_fault(AdmmCtx* ctx, int32_t kind);
int admm_debug_own(AdmmCtx* ctx, int32_t* k8_out, float* theta_h_out);

/* LSTM.forward / init_gate_variables (blocks/lstm.py:43-46, 65-88) without a context.
   x [B,T,D]; wx/wh/wy as above; out_a [B,O].  If gates_out is non-NULL it holds six
   [B,T+1,H] tensors that receive i,f,g,o,c,h at t >= 1 (their time-0 slices are the
   initial state and are read, not written: zero them, or pass c/h as the reference
   does, blocks/lstm.py:69-72); otherwise h_scratch and
   c_scratch ([2,B,H] each) are used.  z_out (may be NULL) receives [4,B*T,H] pre-activations. */
int admm_forward(const float* x, int64_t batch, int32_t seq_len, int32_t input_size,
                 int32_t hidden_size, int32_t output_size,
                 const float* const wx[4], const float* const wh[4], const float* wy,
                 float* const gates_out[6], float* h_scratch, float* c_scratch,
                 float* z_out, float* out_a, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ADMM_LSTM_H */
