#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench/rank_shape.py --n 1048576 --ranks 1,2,4,8 --ipl 4,8 --kernel lds,smem --steps 3 > gpurun_out/rank_shape2.log 2>&1 || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/rank_shape2.log"):
    if l.startswith("{"):
        d = json.loads(l); print(d["P"], d["ipl"], d["kernel"], "%.2f ms" % d["ms_per_step"], "%.3e" % d["predicted_body_updates_per_s"])
PY
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k "virtual or fast" > gpurun_out/pytest_gpu_virtual.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_gpu_virtual.log
