"""Minimal reader for legacy Excel ``.xls`` workbooks (OLE2 compound file + BIFF8 records).

The reference loads ``datasets/GoogleStock/GOOG.xls`` with ``xlrd`` (``dataset.py:392-405``),
which is not available in this environment.  This module reads what that loader uses --
the cell values of the first worksheet -- with the standard library only:

* OLE2 / Compound File Binary: header, DIFAT -> FAT, directory, the ``Workbook`` (or
  ``Book``) stream from regular sectors or the mini stream;
* BIFF8: ``BOUNDSHEET`` (sheet offsets), ``SST`` + ``CONTINUE`` (shared strings), and the
  cell records ``NUMBER``, ``RK``, ``MULRK``, ``LABELSST``, ``FORMULA`` (cached numeric
  result), ``BOOLERR``.

``read_sheet(path, index)`` returns ``{(row, col): value}``; ``cell_value`` mirrors
``xlrd``'s ``sheet.cell_value(row, col)`` for numeric and string cells.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple, Union

_END, _FREE = 0xFFFFFFFE, 0xFFFFFFFF
Cell = Union[float, str, bool]


class XlsError(ValueError):
    """The file is not a BIFF8 workbook this reader understands."""


# ----------------------------------------------------------------------------- OLE2

def _ole_stream(data: bytes, names=('Workbook', 'Book')) -> bytes:
    if data[:8] != bytes.fromhex('d0cf11e0a1b11ae1'):
        raise XlsError('not an OLE2 compound file')
    sec_shift, mini_shift = struct.unpack_from('<HH', data, 0x1E)
    ssz, mssz = 1 << sec_shift, 1 << mini_shift
    n_fat, dir_start = struct.unpack_from('<II', data, 0x2C)
    mini_cutoff, minifat_start, n_minifat, difat_start, n_difat = struct.unpack_from('<IIIII', data, 0x38)

    def sector(i: int) -> bytes:
        off = (i + 1) * ssz
        return data[off:off + ssz]

    difat = list(struct.unpack_from('<109I', data, 0x4C))
    nxt = difat_start
    for _ in range(n_difat):
        if nxt in (_END, _FREE):
            break
        words = struct.unpack(f'<{ssz // 4}I', sector(nxt))
        difat.extend(words[:-1])
        nxt = words[-1]
    fat: List[int] = []
    for s in difat[:n_fat]:
        fat.extend(struct.unpack(f'<{ssz // 4}I', sector(s)))

    def chain(start: int, table: List[int]) -> List[int]:
        out, s, seen = [], start, set()
        while s not in (_END, _FREE) and s < len(table):
            if s in seen:
                raise XlsError('cyclic sector chain')
            seen.add(s)
            out.append(s)
            s = table[s]
        return out

    directory = b''.join(sector(s) for s in chain(dir_start, fat))
    entries = []
    for off in range(0, len(directory), 128):
        e = directory[off:off + 128]
        nlen = struct.unpack_from('<H', e, 0x40)[0]
        name = e[:max(0, nlen - 2)].decode('utf-16-le', errors='replace')
        etype = e[0x42]
        start, size = struct.unpack_from('<II', e, 0x74)
        entries.append((name, etype, start, size))
    root = next((e for e in entries if e[1] == 5), None)
    if root is None:
        raise XlsError('no root entry')
    for want in names:
        for name, etype, start, size in entries:
            if etype != 2 or name != want:
                continue
            if size >= mini_cutoff:
                return b''.join(sector(s) for s in chain(start, fat))[:size]
            ministream = b''.join(sector(s) for s in chain(root[2], fat))
            minifat: List[int] = []
            for s in chain(minifat_start, fat)[:n_minifat or None]:
                minifat.extend(struct.unpack(f'<{ssz // 4}I', sector(s)))
            return b''.join(ministream[m * mssz:(m + 1) * mssz] for m in chain(start, minifat))[:size]
    raise XlsError('no Workbook stream')


# ----------------------------------------------------------------------------- BIFF8

def _records(stream: bytes, pos: int = 0):
    n = len(stream)
    while pos + 4 <= n:
        rtype, rlen = struct.unpack_from('<HH', stream, pos)
        yield pos, rtype, stream[pos + 4:pos + 4 + rlen]
        pos += 4 + rlen


def _rk(v: int) -> float:
    if v & 2:
        x = float(v >> 2 if v < (1 << 31) else (v >> 2) - (1 << 30))
    else:
        x = struct.unpack('<d', struct.pack('<Q', (v & 0xFFFFFFFC) << 32))[0]
    return x / 100.0 if v & 1 else x


class _Chunks:
    """The SST payload with its CONTINUE boundaries (strings restart their encoding flag there)."""

    def __init__(self, parts: List[bytes]):
        self.parts, self.i, self.pos = parts, 0, 0

    def _need(self):
        while self.pos >= len(self.parts[self.i]):
            self.i += 1
            self.pos = 0

    def take(self, n: int) -> bytes:
        out = b''
        while n:
            self._need()
            part = self.parts[self.i]
            k = min(n, len(part) - self.pos)
            out += part[self.pos:self.pos + k]
            self.pos += k
            n -= k
        return out

    def chars(self, count: int, wide: bool) -> str:
        out = []
        while count:
            self._need()
            avail = len(self.parts[self.i]) - self.pos
            if avail == 0:
                continue
            if self.pos == 0 and out:       # continued string: new option byte
                wide = bool(self.take(1)[0] & 1)
                avail -= 1
            w = 2 if wide else 1
            k = min(count, avail // w)
            raw = self.take(k * w)
            out.append(raw.decode('utf-16-le' if wide else 'latin-1'))
            count -= k
        return ''.join(out)


def _sst(parts: List[bytes]) -> List[str]:
    c = _Chunks(parts)
    _total, unique = struct.unpack('<II', c.take(8))
    out = []
    for _ in range(unique):
        cch = struct.unpack('<H', c.take(2))[0]
        flags = c.take(1)[0]
        runs = struct.unpack('<H', c.take(2))[0] if flags & 0x8 else 0
        ext = struct.unpack('<I', c.take(4))[0] if flags & 0x4 else 0
        out.append(c.chars(cch, bool(flags & 1)))
        c.take(4 * runs + ext)
    return out


def read_sheet(path: str, index: int = 0) -> Dict[Tuple[int, int], Cell]:
    """Cells of worksheet `index` (0-based, workbook order) as {(row, col): value}."""
    with open(path, 'rb') as fh:
        stream = _ole_stream(fh.read())
    sheets, sst_parts, in_sst = [], [], False
    for _, rtype, body in _records(stream):
        if rtype == 0x0085:                     # BOUNDSHEET
            sheets.append(struct.unpack_from('<I', body, 0)[0])
        if rtype == 0x00FC:                     # SST
            sst_parts, in_sst = [body], True
            continue
        if rtype == 0x003C and in_sst:          # CONTINUE of SST
            sst_parts.append(body)
            continue
        in_sst = False
        if rtype == 0x000A:                     # EOF of the globals substream
            break
    if index >= len(sheets):
        raise XlsError(f'sheet {index} not found ({len(sheets)} sheets)')
    strings = _sst(sst_parts) if sst_parts else []
    cells: Dict[Tuple[int, int], Cell] = {}
    for _, rtype, body in _records(stream, sheets[index]):
        if rtype == 0x0203:                     # NUMBER
            r, c = struct.unpack_from('<HH', body, 0)
            cells[(r, c)] = struct.unpack_from('<d', body, 6)[0]
        elif rtype == 0x027E:                   # RK
            r, c = struct.unpack_from('<HH', body, 0)
            cells[(r, c)] = _rk(struct.unpack_from('<I', body, 6)[0])
        elif rtype == 0x00BD:                   # MULRK
            r, c0 = struct.unpack_from('<HH', body, 0)
            n = (len(body) - 6) // 6
            for k in range(n):
                cells[(r, c0 + k)] = _rk(struct.unpack_from('<I', body, 4 + 6 * k + 2)[0])
        elif rtype == 0x00FD:                   # LABELSST
            r, c, _, idx = struct.unpack_from('<HHHI', body, 0)
            cells[(r, c)] = strings[idx]
        elif rtype == 0x0006:                   # FORMULA: cached result
            r, c = struct.unpack_from('<HH', body, 0)
            res = body[6:14]
            if res[6:8] != b'\xff\xff':
                cells[(r, c)] = struct.unpack('<d', res)[0]
            elif res[0] == 1:
                cells[(r, c)] = bool(res[2])
        elif rtype == 0x0205:                   # BOOLERR
            r, c = struct.unpack_from('<HH', body, 0)
            if body[7] == 0:
                cells[(r, c)] = bool(body[6])
        elif rtype == 0x000A:                   # EOF of the sheet
            break
    return cells


def cell_value(cells: Dict[Tuple[int, int], Cell], row: int, col: int) -> Cell:
    """xlrd's sheet.cell_value: '' for an empty cell."""
    return cells.get((row, col), '')
