#!/bin/bash
# chunk sweep of the N = 8192 multi-bit CMUX (mb3_3g3) through TFHE_MI355_LARGE_CHUNK
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for c in ${CHUNKS:-384 512 768 1024}; do
  TFHE_MI355_LARGE_CHUNK=$c timeout -k 10 300 python -u bench.py --params mb3_3g3 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r04_mbchunk_$c.log 2>&1 || exit 1
  echo "chunk $c: $(grep '^{' gpurun_out/r04_mbchunk_$c.log | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["value"]))')"
done
