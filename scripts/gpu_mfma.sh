#!/bin/bash
# Experimental MFMA kernel: accuracy/speed probe, then the full GPU round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/mfma_probe.py > gpurun_out/mfma_probe.jsonl 2>&1 || { tail -30 gpurun_out/mfma_probe.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/mfma_probe.jsonl
bash scripts/gpu_round.sh
