#!/bin/bash
# One parameterised GPU recipe (run on the MI355X box through gpurun):
#   bash scripts/gpu.sh <task> [<task> ...]
# tasks (each step under its own time limit; the first failure ends the call):
#   tests[:<pytest -k expr>]  GPU test suite (or a subset; "+" -> space), one process
#   smoke                     __graft_entry__.smoke()
#   bench[:<args>]            bench.py ("+" in <args> becomes a space)
#   prof[:<args>]             rocprofv3 kernel-trace stats of bench.py -> gpurun_out/prof
#   rank[:<args>]             bench/rank_shape.py per-rank emulation ("+" -> space)
#   sweep[:<args>]            bench/sweep.py in-process interleaved A/B
#   rehearsal                 torchrun / self-launch / CLI multi-rank rehearsal on one GPU
#   configs                   bench/configs.py, every BASELINE config
#   pmc[:<bench args>]        three rocprofv3 --pmc passes (kernel-trace only) of bench.py
#   pmcrank[:<rank args>]     the same passes over bench/rank_shape.py
#   trace[:<rank_shape args>] rocprofv3 kernel trace of bench/rank_shape.py + overlap report
#   rankprof[:<rank_shape args>] rocprofv3 kernel-trace stats of bench/rank_shape.py
#   counters                  rocprofv3 -L (the PMC counters this box offers)
#   hash[:<native dir>]       state hashes after 3 steps (scripts/state_hash.py, HASH_CASES)
#   accerr                    per-body error of the sym step path at 4K and 64K (accel_err.py)
#   abtree[:<dir>,<rounds>,<bench args>] alternating bench.py runs of another source tree
#                             (e.g. abv/r3tree: round 3's code) and this one, same box
#   perturb                   smoke() and the 1M accuracy test on a deliberately broken build
#                             (scripts/perturb_build.py -> abv/perturbed): both must FAIL
#   perturb64                 the fp64 512K test and bench --dtype fp64 on abv/perturbed64 (the
#                             fp64 carrier perturbed): both must FAIL
#   ipc                       two-process HIP IPC with / without HSA_ENABLE_IPC_MODE_LEGACY=0
#   span[:<bench args>]       reduce-phase span per step of the default schedule
# Outputs land in gpurun_out/<task>*.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out

args_of() { local a="${1#*:}"; [ "$a" = "$1" ] && a=""; echo "${a//+/ }"; }

step() {  # $1 = limit (s), $2 = log, rest = command
  local lim=$1 log=$2; shift 2
  echo "== $* (limit ${lim}s) -> $log"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  tail -3 "$log"
  if [ $rc -ne 0 ]; then echo "!! rc=$rc: $*"; tail -40 "$log"; exit $rc; fi
}

for task in "$@"; do
  name="${task%%:*}"
  a=$(args_of "$task")
  case "$name" in
    tests)
      if [ -n "${task#tests}" ]; then k="${task#tests:}"; k="${k//+/ }"; else k=""; fi
      step 1500 $out/pytest_gpu${k:+_sel}.log python -u -m pytest tests -x -v -m gpu \
        --timeout 300 --timeout-method thread --durations=30 ${k:+-k "$k"} ;;
    smoke) step 300 $out/smoke.log python __graft_entry__.py smoke ;;
    bench) step 600 $out/bench_$(date +%s).log python bench.py $a ;;
    prof)
      step 600 $out/prof.log rocprofv3 --kernel-trace --stats -d $out/prof -o bench \
        --output-format csv -- python bench.py --steps 3 --warmup 1 $a
      head -6 $out/prof/bench_kernel_stats.csv ;;
    rank) step 1200 $out/rank_$(date +%s).log python bench/rank_shape.py $a ;;
    sweep) step 1200 $out/sweep_$(date +%s).log python bench/sweep.py $a ;;
    rehearsal) step 900 $out/rehearsal.log bash scripts/gpu_torchrun.sh ;;
    configs) step 1200 $out/configs.log python bench/configs.py --md $out/baseline_configs.md ;;
    pmc|pmcrank)
      # pmc: bench.py (+ args); pmcrank: bench/rank_shape.py (+ args), e.g. an fp64 rank shape
      if [ "$name" = pmc ]; then prog="bench.py --steps 2 --warmup 1 --check-samples 0 --phase-steps 0 $a"
      else prog="bench/rank_shape.py $a"; fi
      rm -rf $out/pmc_valu $out/pmc_cycles $out/pmc_lds
      for pass in "valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE" \
                  "cycles SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
                  "lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_SMEM"; do
        set -- $pass; tag=$1; shift
        step 300 $out/pmc_$tag.log rocprofv3 --kernel-trace --pmc "$@" -d $out/pmc_$tag -o pmc \
          --output-format csv -- python $prog
      done
      python scripts/pmc_summary.py > $out/${name}_summary.txt 2>&1; cat $out/${name}_summary.txt ;;
    trace)
      step 600 $out/trace.log rocprofv3 --kernel-trace -d $out/trace -o tr --output-format csv \
        -- python bench/rank_shape.py $a
      t=$(find $out/trace -name "*kernel_trace.csv" | head -1)
      python scripts/overlap_report.py "$t" | tee $out/trace_overlap.txt
      python scripts/trace_steps.py "$t" | tee $out/trace_steps.txt ;;
    rankprof)
      step 900 $out/rankprof.log rocprofv3 --kernel-trace --stats -d $out/rankprof -o rp \
        --output-format csv -- python bench/rank_shape.py $a
      head -8 $out/rankprof/rp_kernel_stats.csv ;;
    counters) step 120 $out/counters.txt rocprofv3 -L ;;
    hash)
      cases=${HASH_CASES:-65536:fp32:auto:1,1048576:fp32:auto:1,65536:fp32:exact:1,524288:fp64:auto:1,65536:fp64:exact:1,262144:fp32:auto:3,262144:fp32:auto:8,1048576:fp32:auto:8}
      tag=$(basename "${a:-in-tree}")
      if [ -n "$a" ]; then  # <a> = another source tree with its own build (e.g. abv/r3tree)
        step 600 $out/hash_$tag.jsonl python -u $a/scripts/state_hash.py --cases $cases
      else
        step 600 $out/hash_$tag.jsonl python -u scripts/state_hash.py --cases $cases
      fi
      cat $out/hash_$tag.jsonl ;;
    abtree)
      IFS=, read -r tree rounds bargs <<< "$a"
      for i in $(seq 1 ${rounds:-2}); do
        for arm in "$tree" .; do
          lab=$([ "$arm" = . ] && echo head || basename "$arm")
          step 600 $out/abtree_${i}_$lab.log python $arm/bench.py --exact-steps 0 \
            --phase-steps 0 --no-replay-audit --no-energy $bargs
          echo "arm=$lab round=$i $(grep -o '"ms_per_step": [0-9.]*' $out/abtree_${i}_$lab.log)" | tee -a $out/abtree.txt
        done
      done ;;
    perturb)
      : > $out/perturb.txt
      for t in smoke scale; do
        if [ $t = smoke ]; then cmd=(python -c "import __graft_entry__ as g; g.smoke()")
        else cmd=(python -u -m pytest tests/test_gpu_scale.py -x -q -k accel_sampled --timeout 300); fi
        timeout -k 10 400 env GRAVSIM_NATIVE_DIR=abv/perturbed "${cmd[@]}" > $out/perturb_$t.log 2>&1
        rc=$?
        echo "perturbed build, $t: rc=$rc (a gate that bites exits non-zero)" | tee -a $out/perturb.txt
        grep -E "AssertionError|assert|error" $out/perturb_$t.log | tail -3 | tee -a $out/perturb.txt
        if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
        if [ $rc -eq 0 ]; then echo "!! the $t gate passed a broken kernel"; exit 1; fi
      done ;;
    accerr)
      step 300 $out/accel_err.txt python -u scripts/accel_err.py --n 4096
      step 300 $out/accel_err_64k.txt python -u scripts/accel_err.py --n 65536
      cat $out/accel_err.txt $out/accel_err_64k.txt ;;
    span)
      # reduce-phase span per step of the default schedule (two runs), same recipe as abfork
      for i in 1 2; do
        d=$out/span_$i; rm -rf $d
        step 600 $d.log rocprofv3 --kernel-trace -d $d -o tr --output-format csv -- python \
          bench.py --steps 6 --warmup 2 --exact-steps 0 --phase-steps 0 --check-samples 0 \
          --no-replay-audit $a
        t=$(find $d -name "*kernel_trace.csv" | head -1)
        echo "default $(python scripts/reduce_span.py $t)" | tee -a $out/span.txt
      done ;;
    perturb64)
      # the fp64 gates on a build whose fp64 x carrier moves by the wrong DPP offset
      # (scripts/perturb_build.py --what carrier64 --out abv/perturbed64): both must FAIL
      : > $out/perturb64.txt
      for t in scale bench; do
        if [ $t = scale ]; then cmd=(python -u -m pytest tests/test_gpu_scale.py -x -q -k fp64_512k --timeout 300)
        else cmd=(python bench.py --dtype fp64 --n 524288 --steps 2 --warmup 1 --exact-steps 0 --phase-steps 0 --no-replay-audit --no-energy); fi
        timeout -k 10 400 env GRAVSIM_NATIVE_DIR=abv/perturbed64 "${cmd[@]}" > $out/perturb64_$t.log 2>&1
        rc=$?
        echo "perturbed fp64 build, $t: rc=$rc (a gate that bites exits non-zero)" | tee -a $out/perturb64.txt
        grep -E "AssertionError|assert|work_audit|error" $out/perturb64_$t.log | tail -3 | cut -c1-400 | tee -a $out/perturb64.txt
        if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit $rc; fi
        if [ $rc -eq 0 ]; then echo "!! the fp64 $t gate passed a broken kernel"; exit 1; fi
      done ;;
    ipc)
      # two-process HIP IPC (memory + event) with the launcher's dmabuf setting and without it
      step 300 $out/ipc_dmabuf.log env HSA_ENABLE_IPC_MODE_LEGACY=0 python tests/ipc_peer.py pair
      step 300 $out/ipc_legacy.log env -u HSA_ENABLE_IPC_MODE_LEGACY python tests/ipc_peer.py pair ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
