set -e
for v in "$@"; do echo "== kbench$v"; timeout -k 5 60 ./tools/kbench$v 8192 s3; done
