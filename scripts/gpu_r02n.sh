#!/bin/bash
# host-pointer ABI probe: fresh / reused / pinned buffers, with and without torch's HIP context
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02n
rm -f gpurun_out/r02n/probe.log
timeout -k 10 200 python scripts/probes/host_abi_probe.py >> gpurun_out/r02n/probe.log 2>&1 || exit $?
PROBE_TORCH=1 timeout -k 10 200 python scripts/probes/host_abi_probe.py >> gpurun_out/r02n/probe.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02n/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r02n/probe.log
grep -o '"host_abi": {"value": [0-9.]*' gpurun_out/r02n/bench.log
