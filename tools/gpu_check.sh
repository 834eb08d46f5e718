#!/bin/bash
# One GPU-box session: microbench, smoke, GPU parity tests, bench, rocprof.
# Every GPU step has its own time limit; a crash (not a test failure) stops
# the script.  Output goes to gpurun_out/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

STEPS="${STEPS:-ubench smoke pytest bench prof}"
for s in $STEPS; do
  case $s in
    ubench) step ubench 120 ./tools/ubench_int || exit 3 ;;
    ubdep) step ubdep 300 ./tools/ubench_dep || exit 3 ;;
    ubissue) step ubissue 300 ./tools/ubench_issue || exit 3 ;;
    smoke) step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    pytest) step pytest 1200 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider -rA --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"}; rc=$?; ok_or_testfail $rc || exit 3 ;;
    pytestf) step pytestf 1200 python3 -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -x -p no:cacheprovider -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}; rc=$?; ok_or_testfail $rc || exit 3 ;;
    bench) step bench 600 python3 -u bench.py ${BENCH_ARGS:-} || exit 3 ;;
    configsab)  # the same configs with knob settings alternated: CONFIGS_AB="k=v1 k=v2", CONFIGS_ROUNDS rounds
      for r in $(seq ${CONFIGS_ROUNDS:-2}); do
        for kv in ${CONFIGS_AB}; do
          step "configsab_${kv}_r$r" 600 python3 -u tools/bench_configs.py ${CONFIGS_ARGS:-decode} --knob $kv || exit 3
        done
      done ;;
    configs) step configs 900 python3 -u tools/bench_configs.py ${CONFIGS_ARGS:-u64 decode host sweep --cpu} || exit 3 ;;
    prof)
      export TMPDIR=/tmp
      step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 1 --cpu-sample 0 || exit 3 ;;
    dist2) step dist2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --ids-per-gpu 2e8 --cpu-sample 0 || exit 3 ;;
    dist2full) step dist2full 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-sample 0 || exit 3 ;;
    dist4full) step dist4full 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 4 --steps 3 --warmup 1 --cpu-sample 0 || exit 3 ;;
    roots) step roots 300 python3 -u tools/bench_roots.py ${ROOTS_ARGS:-} || exit 3
           step profroots 120 ./tools/prof_roots 32 300 || exit 3 ;;
    abenc) step abenc 600 python3 -u tools/ab_encode.py ${ABENC_ARGS:-} || exit 3 ;;
    abenc2) step abenc2 600 python3 -u tools/ab_encode.py ${ABENC2_ARGS:-} || exit 3 ;;
    abenc3) step abenc3 600 python3 -u tools/ab_encode.py ${ABENC3_ARGS:-} || exit 3 ;;
    abflows) step abflows 600 python3 -u tools/ab_flows.py ${ABFLOWS_ARGS:-} || exit 3 ;;
    profabflows)
      export TMPDIR=/tmp
      step profabflows 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profabflows" -o run -- python3 "$ROOT/tools/ab_flows.py" ${PROFAB_ARGS:---modes 1 --rounds 2} || exit 3 ;;
    dist4) step dist4 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 3 --warmup 1 --ids-per-gpu 1e8 --cpu-sample 0 || exit 3 ;;
    tune) step tune 600 ./tools/tune_encode ${TUNE_ARGS:-} || exit 3 ;;
    tunebsgs) step tunebsgs 600 ./tools/tune_bsgs ${TUNE_ARGS:-} || exit 3 ;;
    listctr) step listctr 120 rocprofv3 -L || true ;;
    pmcsq)
      export TMPDIR=/tmp
      step pmcsq 600 rocprofv3 --pmc ${PMC_SQ:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} --output-format csv -d "$OUT/pmcsq" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 || exit 3 ;;
    proflows)
      export TMPDIR=/tmp
      step proflows 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proflows" -o run -- python3 "$ROOT/tools/bench_configs.py" flows packets --steps 4 || exit 3 ;;
    proftrace)  # kernel + memory-copy + HIP runtime trace (no counters) of one command, for the gaps between them
      export TMPDIR=/tmp
      step proftrace 600 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --stats --output-format csv -d "$OUT/proftrace" -o run -- python3 "$ROOT/tools/bench_configs.py" ${PROFTRACE_ARGS:-decode --rt-modes 2} --steps 10 || exit 3 ;;
    profcfg)  # kernel stats for the secondary configs' kernels (u64 encode, u32/u64 root test)
      export TMPDIR=/tmp
      step profcfg 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profcfg" -o run -- python3 "$ROOT/tools/bench_configs.py" ${PROFCFG_ARGS:-u64 decode decode64} --steps 10 || exit 3 ;;
    pmccfg)  # FETCH_SIZE and SQ passes over the same configs, one counter group per run
      export TMPDIR=/tmp
      step pmccfg_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmccfg_fetch" -o run -- python3 "$ROOT/tools/bench_configs.py" ${PROFCFG_ARGS:-u64 decode decode64} --steps 2 || exit 3
      step pmccfg_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmccfg_sq" -o run -- python3 "$ROOT/tools/bench_configs.py" ${PROFCFG_ARGS:-u64 decode decode64} --steps 2 || exit 3 ;;
    decshape) step decshape 600 python3 -u tools/bench_decode.py ${DECSHAPE_ARGS:-} || exit 3 ;;
    tuneu64) step tuneu64 600 ./tools/tune_u64 || exit 3 ;;
    flowsbench) step flowsbench 600 python3 -u tools/bench_configs.py flows --steps 6 || exit 3 ;;
    dec64)  # u64 root test: BSGS (default) vs Horner
      step dec64_bsgs 300 python3 -u tools/bench_configs.py decode64 --steps 10 --cpu || exit 3
      step dec64_horner 300 python3 -u tools/bench_configs.py decode64 --steps 10 --knob rt64_horner=1 || exit 3 ;;
    fig2)  # the reference's figure-2 command lines against the drop-in programs (host and --gpu)
      step fig2_host 600 python3 -u tools/run_fig2.py "$OUT/fig2_host" --trials 100 || exit 3
      step fig2_gpu 600 python3 -u tools/run_fig2.py "$OUT/fig2_gpu" --trials 20 --gpu || exit 3 ;;
    dist2rccl)  # two ranks through the native RCCL communicator (on one GPU if that is all there is)
      NCCL_DEBUG=WARN step dist2rccl 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 2 --steps 3 --warmup 1 --ids-per-gpu 1e8 --cpu-sample 0 || exit 3 ;;
    passes)  # u32 t > 80: BSGS passes (default) vs the power chain
      step sweep_passes 300 python3 -u tools/bench_configs.py sweep --steps 6 || exit 3
      step sweep_chain 300 python3 -u tools/bench_configs.py sweep --steps 6 --knob u32_passes=0 || exit 3 ;;
    pmc)
      export TMPDIR=/tmp
      step pmc 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 || exit 3 ;;
  esac
done
echo ALLDONE | tee -a "$OUT/steps.log"
