#!/bin/bash
# Multi-rank rehearsal on a ONE-GPU box: every rank runs on device 0 and RCCL connects the
# ranks through its socket transport (GRAVSIM_RCCL_RANK_HOSTS=1 gives each rank its own
# NCCL_HOSTID, gravsim/parallel/comm.py). Checks the torchrun launch contract of bench.py
# (one JSON line, max over ranks) and the CLI (--nproc, dumps, checkpoints, resume across
# rank counts). Throughput here is meaningless (loopback sockets, one shared GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tr
export TMPDIR=/tmp GRAVSIM_RCCL_RANK_HOSTS=1
out=gpurun_out/tr
run="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
# bench.py without a launcher starts its own ranks (parallel/launch.py)
timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 1 --n 65536 > $out/bench2_self.log 2>&1 \
  || { tail -30 $out/bench2_self.log; exit 1; }
grep '^{' $out/bench2_self.log
timeout -k 10 240 $run --nproc-per-node 2 --master-port 29611 bench.py --gpus 2 --steps 3 \
  --warmup 1 --num-bodies 65536 > $out/bench2.log 2>&1 || { tail -30 $out/bench2.log; exit 1; }
grep '^{' $out/bench2.log
timeout -k 10 240 $run --nproc-per-node 4 --master-port 29612 bench.py --gpus 4 --steps 2 \
  --warmup 1 --num-bodies 131072 > $out/bench4.log 2>&1 || { tail -30 $out/bench4.log; exit 1; }
grep '^{' $out/bench4.log
timeout -k 10 240 $run --nproc-per-node 2 --master-port 29613 bench.py --gpus 2 --steps 2 \
  --warmup 1 --num-bodies 65536 --strategy ring --mode split > $out/bench2_ring.log 2>&1 \
  || { tail -30 $out/bench2_ring.log; exit 1; }
grep '^{' $out/bench2_ring.log
# The driver's N=8 shape: bench.py --gpus 8 at the headline N = 1M, 8 ranks sharing this GPU
# (RCCL over loopback sockets; throughput meaningless, the contract and the path are not).
timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 --n 1048576 > $out/bench8_1m.log 2>&1 \
  || { tail -30 $out/bench8_1m.log; exit 1; }
grep '^{' $out/bench8_1m.log
# CLI: 2 ranks (sym, checkpoint every 3) vs 1 rank, then a 1-rank resume of the 2-rank
# checkpoint, plus 3 and 8 ranks (3: uneven row blocks, 3/3/2 of 8); the final dumps must be
# identical text, and every multi-rank run must report the gated overlap (3), the
# segmented step graph and a clean work audit in its metrics line.
common="--n 40000 --device gpu --mode sym --log-format none --quiet"
rm -f $out/m*.json
timeout -k 10 240 python -m gravsim $common --steps 6 --nproc 2 --dump $out/p2.txt \
  --checkpoint-dir $out/ck --checkpoint-every 3 --metrics-json $out/m2.json --diagnostics > $out/cli2.log 2>&1 \
  || { tail -30 $out/cli2.log; exit 1; }
timeout -k 10 240 python -m gravsim $common --steps 6 --dump $out/p1.txt \
  > $out/cli1.log 2>&1 || { tail -30 $out/cli1.log; exit 1; }
timeout -k 10 240 python -m gravsim $common --steps 6 --nproc 3 --dump $out/p3.txt \
  --metrics-json $out/m3.json --diagnostics > $out/cli3.log 2>&1 || { tail -30 $out/cli3.log; exit 1; }
timeout -k 10 300 python -m gravsim $common --steps 6 --nproc 8 --dump $out/p8.txt \
  --metrics-json $out/m8.json --diagnostics > $out/cli8.log 2>&1 || { tail -30 $out/cli8.log; exit 1; }
ck3=$(ls $out/ck/*00000003* | head -1)
timeout -k 10 240 python -m gravsim $common --steps 3 --resume "$ck3" --dump $out/pr.txt \
  > $out/clir.log 2>&1 || { tail -30 $out/clir.log; exit 1; }
cmp $out/p1.txt $out/p2.txt && cmp $out/p1.txt $out/p3.txt && cmp $out/p1.txt $out/p8.txt \
  && cmp $out/p1.txt $out/pr.txt \
  && echo "CLI dumps identical (P=1, 2, 3, 8; P=2 ckpt -> P=1 resume)" || exit 1
python - $out/m2.json $out/m3.json $out/m8.json <<'PY' || exit 1
import json, sys
e0 = None
for f in sys.argv[1:]:
    m = json.loads(open(f).read().splitlines()[-1])
    e = m["extra"]
    print(f, "nranks", m["nranks"], "overlap", e["overlap"], "graph", e["graph"],
          "segments", e["graph_segments"], "work_audit", e["work_audit"])
    assert e["overlap"] == 3 and e["graph"] == "segmented" and e["work_audit"] == "ok", e
    c = e["conservation"]
    print("   energy", c["energy_start"], "->", c["energy_end"], "momentum drift",
          c["momentum_rel_drift"])
    e0 = c["energy_start"] if e0 is None else e0
    assert abs(c["energy_start"] - e0) <= 1e-10 * abs(e0), (c["energy_start"], e0)
PY
