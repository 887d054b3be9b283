#!/bin/bash
# Named GPU-box steps (from the repo root, via gpurun): bash tools/gpu_steps.sh <tag> <step>...
# (The one-off round scripts of rounds 1-5 are folded into these steps; tools/gpu_run.sh runs
# ad-hoc '<name>|<seconds>|<command>' steps the same way.)
#   tests  — pytest -m gpu;  smoke — __graft_entry__.smoke();  bench — default bench.py;
#   load26 — RMAT-26 generate + load + GO leg only (load time);  prof26 — kernel trace of the bench;
#   pmc26 / pmc22 / sq26 — GO HBM / SQ counters;  pmcsp — SHORTEST (rolling + one-pair) HBM and SQ
#   counters;  pmcc5 — C5 GO 4 STEPS HBM counters and kernel trace;  bench8 — 8-rank rehearsal
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for step in "$@"; do
  case $step in
    tests)
      NBG_COMM_TIMEOUT_S=60 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; } ;;
    configs)
      timeout -k 10 1100 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 1200 --timeout-method thread \
        > "$OUT/pytest_configs.log" 2>&1 || { tail -40 "$OUT/pytest_configs.log"; exit 1; } ;;
    load26)
      timeout -k 10 900 python -u bench.py --scale 26 --roots 16 --steps 2 --sp-pairs 0 --no-cpu-baseline \
        --c5-scale 0 --getbound-reqs 0 --no-profile > "$OUT/load26.json" 2> "$OUT/load26.log" \
        || { tail -30 "$OUT/load26.log"; exit 1; } ;;
    pmc26|pmc22)
      sc=${step#pmc}
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 400 rocprofv3 --pmc $c -d "$OUT/pmc${sc}_$c" -o run --output-format csv -- \
          python3 -u bench.py --scale $sc --steps 1 --warmup 1 --sp-pairs 0 --no-cpu-baseline --no-profile \
          --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 > "$OUT/pmc${sc}_$c.json" 2> "$OUT/pmc${sc}_$c.log" \
          || { tail -30 "$OUT/pmc${sc}_$c.log"; exit 1; }
      done
      python3 tools/pmc_summary.py $(find "$OUT/pmc${sc}_FETCH_SIZE" "$OUT/pmc${sc}_WRITE_SIZE" -name '*counter_collection.csv') \
        > "$OUT/pmc_hbm_rmat${sc}.json" ;;
    sq26)   # where the final step's waves spend their cycles (one SQ pass, 8 counters)
      c="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
      timeout -s KILL 400 rocprofv3 --pmc $c -d "$OUT/sq26" -o run --output-format csv -- \
        python3 -u bench.py --steps 1 --warmup 1 --sp-pairs 0 --no-cpu-baseline --no-profile \
        --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 > "$OUT/sq26.json" 2> "$OUT/sq26.log" \
        || { tail -30 "$OUT/sq26.log"; exit 1; }
      python3 tools/pmc_summary.py $(find "$OUT/sq26" -name '*counter_collection.csv') > "$OUT/pmc_sq_rmat26.json" ;;
    pmcsp)   # SHORTEST kernels (rolling k_ch_roll<4>, one-pair k_ch_step<1>): HBM bytes and SQ cycles
      i=0
      for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"; do
        i=$((i + 1))
        PROBE_ROUNDS=1 timeout -s KILL 400 rocprofv3 --pmc $c -d "$OUT/pmcsp_$i" -o run --output-format csv -- \
          python3 -u tools/sp_batch_probe.py 26 2000 default > "$OUT/pmcsp_$i.txt" 2>&1 \
          || { tail -30 "$OUT/pmcsp_$i.txt"; exit 1; }
      done
      python3 tools/pmc_summary.py $(find "$OUT/pmcsp_1" "$OUT/pmcsp_2" -name '*counter_collection.csv') \
        > "$OUT/pmc_hbm_sp_rmat26.json"
      python3 tools/pmc_summary.py $(find "$OUT/pmcsp_3" -name '*counter_collection.csv') > "$OUT/pmc_sq_sp_rmat26.json" ;;
    pmcc5)   # C5 GO 4 STEPS OVER knows, likes (RMAT-24): HBM bytes per kernel
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 400 rocprofv3 --pmc $c -d "$OUT/pmcc5_$c" -o run --output-format csv -- \
          python3 -u tools/c5_probe.py 24 2 > "$OUT/pmcc5_$c.txt" 2>&1 || { tail -30 "$OUT/pmcc5_$c.txt"; exit 1; }
      done
      python3 tools/pmc_summary.py $(find "$OUT/pmcc5_FETCH_SIZE" "$OUT/pmcc5_WRITE_SIZE" -name '*counter_collection.csv') \
        > "$OUT/pmc_hbm_c5_rmat24.json"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/profc5" -o run --output-format csv -- \
        python3 -u tools/c5_probe.py 24 2 > "$OUT/profc5.txt" 2>&1 || { tail -30 "$OUT/profc5.txt"; exit 1; } ;;
    prof26)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof26" -o run --output-format csv -- \
        python3 -u bench.py --sp-pairs 2000 --no-cpu-baseline --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 \
        > "$OUT/bench_prof26.json" 2> "$OUT/bench_prof26.log" || { tail -30 "$OUT/bench_prof26.log"; exit 1; } ;;
    go26|go26flags)
      [ "$step" = go26flags ] && export NBG_MARK_FLAGS=1
      timeout -k 10 600 python -u bench.py --sp-pairs 0 --no-cpu-baseline --verify 4 --c2 0 --c5-scale 0 \
        --getbound-reqs 0 > "$OUT/$step.json" 2> "$OUT/$step.log" || { tail -30 "$OUT/$step.log"; exit 1; }
      unset NBG_MARK_FLAGS ;;
    anat26)   # GO 3 STEPS per-query anatomy, kernel-traced
      timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT/anat26" -o run --output-format csv -- \
        python3 -u tools/mark_probe.py 26 16 > "$OUT/anat26.txt" 2>&1 || { tail -30 "$OUT/anat26.txt"; exit 1; } ;;
    wake)   # host wake-up after a query's last kernel: event poll vs mapped-flag poll
      timeout -k 10 120 ./tools/wake_probe > "$OUT/wake.txt" 2>&1 || { tail -30 "$OUT/wake.txt"; exit 1; } ;;
    wakeab)   # GO leg and small legs with the flag wake-up vs the event wait
      timeout -k 10 700 bash tools/go_ab.sh "$TAG/wakeab" nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_WAKE=event \
        > "$OUT/wakeab.txt" 2>&1 || { tail -30 "$OUT/wakeab.txt"; exit 1; }
      for wk in flag event; do
        NBG_WAKE=$wk timeout -k 10 400 python -u bench.py --scale 16 --roots 4 --steps 1 --warmup 1 --sp-pairs 0 \
          --c2 0 --c5-scale 0 --c1-reqs 3000 --getbound-reqs 2000 --verify 0 --no-profile --no-cpu-baseline \
          > "$OUT/small_$wk.json" 2> "$OUT/small_$wk.log" || { tail -30 "$OUT/small_$wk.log"; exit 1; }
      done ;;
    spwake)   # SHORTEST latency with the flag wake-up vs the event wait
      timeout -k 10 1000 bash tools/sp_ab.sh "$TAG/spwake" nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_WAKE=event \
        > "$OUT/spwake.txt" 2>&1 || { tail -30 "$OUT/spwake.txt"; exit 1; } ;;
    goprev)   # GO leg: this build vs nebula_amd/libnbg_prev.so (the previous commit's)
      timeout -k 10 700 bash tools/go_ab.sh "$TAG/goprev" nebula_amd/libnbg.so nebula_amd/libnbg_prev.so \
        > "$OUT/goprev.txt" 2>&1 || { tail -30 "$OUT/goprev.txt"; exit 1; } ;;
    smallab)   # the small legs: this build vs nebula_amd/libnbg_prev.so, two rounds
      for round in 1 2; do
        for lib in libnbg libnbg_prev; do
          NBG_LIB=$PWD/nebula_amd/$lib.so NBG_GN_TRACE=1 timeout -k 10 400 python -u bench.py --scale 16 --roots 4 --steps 1 \
            --warmup 1 --sp-pairs 0 --c2 0 --c5-scale 0 --c1-reqs 3000 --getbound-reqs 2000 --verify 0 --no-profile \
            --no-cpu-baseline > "$OUT/small_${lib}_r$round.json" 2> "$OUT/small_${lib}_r$round.log" \
            || { tail -30 "$OUT/small_${lib}_r$round.log"; exit 1; }
          python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['getbound']; c=d['c1_nba']; print(sys.argv[2], 'getBound p50', round(g['p50_ms'],4), 'p90', round(g['p90_ms'],4), 'C1 p50', round(c['p50_ms'],4), 'C ABI', round(c['c_abi_p50_ms'],4))" "$OUT/small_${lib}_r$round.json" "$lib" | tee -a "$OUT/smallab.txt"
        done
      done ;;
    gnteam)   # getBound: the encoding team size (NBG_GN_THREADS), two rounds
      for round in 1 2; do
        for tm in 0 2 4 8; do
          NBG_GN_THREADS=$tm NBG_GN_TRACE=1 timeout -k 10 400 python -u bench.py --scale 16 --roots 4 --steps 1 \
            --warmup 1 --sp-pairs 0 --c2 0 --c5-scale 0 --c1-reqs 0 --getbound-reqs 2000 --verify 0 --no-profile \
            --no-cpu-baseline > "$OUT/gn_t${tm}_r$round.json" 2> "$OUT/gn_t${tm}_r$round.log" \
            || { tail -30 "$OUT/gn_t${tm}_r$round.log"; exit 1; }
          python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['getbound']; print('threads', sys.argv[2], 'getBound p50', round(g['p50_ms'],4), 'p90', round(g['p90_ms'],4))" "$OUT/gn_t${tm}_r$round.json" "$tm" | tee -a "$OUT/gnteam.txt"
          grep 'gn trace' "$OUT/gn_t${tm}_r$round.log" | tail -1 | tee -a "$OUT/gnteam.txt"
        done
      done ;;
    spprev)   # SHORTEST: this build vs nebula_amd/libnbg_prev.so
      timeout -k 10 1000 bash tools/sp_ab.sh "$TAG/spprev" nebula_amd/libnbg.so nebula_amd/libnbg_prev.so \
        > "$OUT/spprev.txt" 2>&1 || { tail -30 "$OUT/spprev.txt"; exit 1; } ;;
    ptest)
      timeout -k 10 400 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_configs.py -x -v --timeout 300 \
        --timeout-method thread > "$OUT/pytest_path.log" 2>&1 || { tail -40 "$OUT/pytest_path.log"; exit 1; } ;;
    sp26|sp26host)
      [ "$step" = sp26host ] && export NBG_SP_MODE=host
      timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-profile --no-cpu-baseline --verify 4 --c2 0 \
        --c5-scale 0 --getbound-reqs 0 > "$OUT/$step.json" 2> "$OUT/$step.log" || { tail -30 "$OUT/$step.log"; exit 1; }
      unset NBG_SP_MODE ;;
    probe22|probe26)
      sc=${step#probe}
      timeout -k 10 300 python -u tools/sp_probe.py $sc 4000 > "$OUT/$step.txt" 2>&1 \
        || { tail -30 "$OUT/$step.txt"; exit 1; }
      NBG_SP_MODE=host timeout -k 10 300 python -u tools/sp_probe.py $sc 4000 > "$OUT/${step}_legacy.txt" 2>&1 \
        || { tail -30 "$OUT/${step}_legacy.txt"; exit 1; } ;;
    spprof26)   # kernel trace of the one-pair SP queries (default path)
      timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT/spprof26" -o run --output-format csv -- \
        python3 -u tools/sp_probe.py 26 400 > "$OUT/spprof26.txt" 2>&1 || { tail -30 "$OUT/spprof26.txt"; exit 1; } ;;
    kpad)   # SHORTEST chain length A/B: one launch fewer / more than the sized chain
      timeout -k 10 1000 bash tools/sp_ab.sh "$TAG/kpad" nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_KPAD=-1 \
        nebula_amd/libnbg.so,NBG_SP_KPAD=1 > "$OUT/kpad.txt" 2>&1 || { tail -30 "$OUT/kpad.txt"; exit 1; } ;;
    spgrid)   # SHORTEST step-grid A/B
      timeout -k 10 1100 bash tools/sp_ab.sh "$TAG/spgrid" nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_GRID=128 \
        nebula_amd/libnbg.so,NBG_SP_GRID=512 > "$OUT/spgrid.txt" 2>&1 || { tail -30 "$OUT/spgrid.txt"; exit 1; } ;;
    small)   # the small-request legs (C1 nba, getBound) with the getBound phase trace
      NBG_GN_TRACE=1 timeout -k 10 400 python -u bench.py --scale 16 --roots 4 --steps 1 --warmup 1 --sp-pairs 0 \
        --c2 0 --c5-scale 0 --c1-reqs 3000 --getbound-reqs 2000 --verify 0 --no-profile \
        > "$OUT/small.json" 2> "$OUT/small.log" || { tail -30 "$OUT/small.log"; exit 1; } ;;
    smallprof)   # kernel trace of the small-request legs
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/smallprof" -o run --output-format csv -- \
        python3 -u bench.py --scale 16 --roots 4 --steps 1 --warmup 1 --sp-pairs 0 --c2 0 --c5-scale 0 \
        --c1-reqs 2000 --getbound-reqs 2000 --verify 0 --no-profile --no-cpu-baseline \
        > "$OUT/smallprof.json" 2> "$OUT/smallprof.log" || { tail -30 "$OUT/smallprof.log"; exit 1; } ;;
    p8)   # the 8-way partition, in-process ranks on one GPU
      NBG_COMM_TIMEOUT_S=60 timeout -k 10 900 python -u -m pytest tests/test_gpu_partition8.py -x -v --timeout 150 --timeout-method thread \
        > "$OUT/pytest_partition8.log" 2>&1 || { tail -40 "$OUT/pytest_partition8.log"; exit 1; } ;;
    rccl8)   # 8 RCCL processes on one GPU (socket transport)
      timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py --same-device > "$OUT/rccl8_probe.log" 2>&1 \
        || { tail -40 "$OUT/rccl8_probe.log"; exit 1; } ;;
    bench8)   # 8-rank bench rehearsal on one GPU (RMAT-20, socket transport)
      NBG_SAME_DEVICE=1 timeout -k 10 900 python -u bench.py --gpus 8 --scale 20 --sp-pairs 2000 --steps 3 --warmup 1 \
        > "$OUT/bench8_rmat20_same_device.json" 2> "$OUT/bench8.log" || { tail -40 "$OUT/bench8.log"; exit 1; } ;;
    diagnba)   # FindPathTest goldens over 8 / 7 in-process ranks, per case and mode
      NBG_COMM_TIMEOUT_S=60 timeout -k 10 300 python -u tools/diag_nba_paths.py 8 7 > "$OUT/diag_nba_paths.txt" 2>&1 \
        || { tail -30 "$OUT/diag_nba_paths.txt"; exit 1; } ;;
    pytest:*)   # one test file or node id (a hang dumps every thread's stack at 150 s, before the
                # box's 180 s silence limit; collectives give up after NBG_COMM_TIMEOUT_S)
      t=${step#pytest:}; n=$(basename "${t%%::*}" .py)
      NBG_COMM_TIMEOUT_S=${NBG_COMM_TIMEOUT_S:-60} timeout -k 10 900 python -u -m pytest "$t" -x -v --timeout 150 --timeout-method thread \
        > "$OUT/pytest_$n.log" 2>&1 || { tail -40 "$OUT/pytest_$n.log"; exit 1; } ;;
    bench)
      timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; } ;;
  esac
  echo "step $step done"
done
