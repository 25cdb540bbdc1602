#!/bin/bash
# The one GPU-box recipe (run through gpurun from the repo root):
#
#   bash tools/gpu_round.sh TAG STEP [STEP ...]
#
#   tests            pytest -m gpu (all), -v, per-test timeout
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench:CONFIG     python bench.py --config CONFIG        -> bench_CONFIG.json
#   pmc:CONFIG       K1 HBM bytes: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE
#                    (separate passes) over tools/k1_once.py CONFIG
#                    -> pmc_CONFIG.json (config + build id stamped)
#   sq:CONFIG        K1 SQ instruction / wait counters, one pass -> sq_CONFIG.json
#   sq2:CONFIG       K1 SQ active-per-pipe / waitcnt counters -> sq2_CONFIG.json
#   prof:CONFIG      rocprofv3 --kernel-trace --stats of a bench run
#                    -> kernel_stats_CONFIG.csv + the bench line under it
#   timeline:SHARD   kernel trace of repeated C3 shard steps -> per-kernel durations and gaps
#   shards:W         tools/shard_step.py: per-rank step of a W-way C3 split
#   e2ecold:CONFIG   tools/e2e_cold.py: first drop-in call of a fresh process (+ phases)
#   e2esweep:CONFIG:K=V,..;..  e2ecold per runtime setting (fresh process each)
#   mp:CONFIG[:BASES]  bench.py --path maxpairs (F2, reference emission order)
#   mpprof:CONFIG[:BASES] rocprofv3 --kernel-trace --stats of that run
#   f3:CONFIG[:BASES]  bench.py --path lcpitv (F3, intervals + visitor events)
#   f3prof:CONFIG[:BASES] rocprofv3 --kernel-trace --stats of that run
#   llvstats         tools/llv_window_stats.py c3 and c5 (.llv values per K1 window)
#   rehearse:W[:BASES]  bench.py --gpus W as W ranks on this one GPU (gloo staging)
#   pmcablate:V,...  K1 SQ counters under GT_SMAX_DEBUG ablation bits at C3
#   fetchablate:V,... K1 FETCH_SIZE under GT_SMAX_DEBUG ablation bits at C3
#   tilestats:CONFIG tools/tile_stats.py (active segments and records per K1 tile)
#   abm:KIND:BASES:MINLEN:SHARD:LIB,... the in-tree library and several others, one process
#   ab:LIB:KIND:BASES:MINLEN:SHARD   A/B of the in-tree library against LIB
#                    (tools/ab_interleave.py, 8 interleaved rounds)
#
# Outputs go to gpurun_out/TAG/ (profiler databases are summarised and then
# removed: gpurun copies back at most 64 MiB).  Every GPU step runs under its own timeout
# and the script stops at the first failure (set -e).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
# the diagnostic build of the library (GT_SMAX_DEBUG / GT_SMAX_STAMPS exist
# only there): make -C genometools_smax_amd builds it beside the production one
DIAGLIB=$R/genometools_smax_amd/lib/diag/libgtsmax_hip.so
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
SQ2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
for S in "$@"; do
  echo "[gpu_round] $S $(date +%T)"
  case $S in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
        > "$O/gpu_tests.log" 2>&1 ;;
    tests:*)
      K=${S#tests:}
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
        -k "$K" > "$O/gpu_tests_sel.log" 2>&1 ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench:*)
      C=${S#bench:}
      timeout -k 10 900 python -u bench.py --config "$C" > "$O/bench_$C.json" 2> "$O/bench_$C.err" ;;
    pmc:*)
      C=${S#pmc:}
      for X in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $X --kernel-include-regex smax_scan_kernel \
          -d "$O/pmc_${C}_$X" -o p -- python3 "$R/tools/k1_once.py" "$C" 5 > "$O/pmc_${C}_$X.log" 2>&1)
      done
      python3 tools/rocpd_summary.py pmc "$O/pmc_$C.json" smax_scan_kernel "$C" \
        "$O/pmc_${C}_FETCH_SIZE/p_results.db" "$O/pmc_${C}_WRITE_SIZE/p_results.db"
      rm -rf "$O/pmc_${C}_FETCH_SIZE" "$O/pmc_${C}_WRITE_SIZE" ;;
    sq2:*)
      # where the waves' cycles go: parked in s_waitcnt, issuing per pipe
      C=${S#sq2:}
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $SQ2 --kernel-include-regex smax_scan_kernel \
        -d "$O/sq2_$C" -o p -- python3 "$R/tools/k1_once.py" "$C" 5 > "$O/sq2_$C.log" 2>&1)
      python3 tools/rocpd_summary.py pmc "$O/sq2_$C.json" smax_scan_kernel "$C" "$O/sq2_$C/p_results.db"
      rm -rf "$O/sq2_$C" ;;
    sq:*)
      C=${S#sq:}
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex smax_scan_kernel \
        -d "$O/sq_$C" -o p -- python3 "$R/tools/k1_once.py" "$C" 5 > "$O/sq_$C.log" 2>&1)
      python3 tools/rocpd_summary.py pmc "$O/sq_$C.json" smax_scan_kernel "$C" "$O/sq_$C/p_results.db"
      rm -rf "$O/sq_$C" ;;
    prof:*)
      C=${S#prof:}
      (cd /tmp && TMPDIR=/tmp timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof_$C" -o p -- \
        python3 "$R/bench.py" --config "$C" --steps 20 --warmup 3 --no-cpu-baseline --no-end-to-end \
        > "$O/prof_bench_$C.json" 2> "$O/prof_bench_$C.err")
      python3 tools/rocpd_summary.py stats "$O/prof_$C/p_results.db" "$O/kernel_stats_$C.csv"
      rm -rf "$O/prof_$C" ;;
    ab:*)
      # ab:LIBB:CONFIGKIND:BASES:MINLEN:SHARD -- tools/ab_interleave.py, in-tree
      # library (A) against LIBB (B) in one process, interleaved rounds
      IFS=: read -r _ LIBB KIND BASES MINLEN SHARD <<< "$S"
      timeout -k 10 600 python -u tools/ab_interleave.py "$KIND" "$BASES" "$MINLEN" "$LIBB" 8 "$SHARD" \
        > "$O/ab_${KIND}_${SHARD//\//of}_vs_$(basename "$(dirname "$LIBB")").txt" 2>&1 ;;
    abm:*)
      # abm:KIND:BASES:MINLEN:SHARD:LIB[,LIB...] -- tools/ab_multi.py, the in-tree
      # library and each LIB in one process, rotated rounds
      IFS=: read -r _ KIND BASES MINLEN SHARD LIBS <<< "$S"
      timeout -k 10 600 python -u tools/ab_multi.py "$KIND" "$BASES" "$MINLEN" "$SHARD" 8 ${LIBS//,/ } \
        > "$O/abm_${KIND}_${SHARD//\//of}.txt" 2>&1 ;;
    ablate:*)
      # ablate:V1,V2,...  K1 time under GT_SMAX_DEBUG ablation bits at C3 (diag build)
      GT_SMAX_LIB=$DIAGLIB timeout -k 10 600 python -u tools/k1_ablate.py human 3e9 "${S#ablate:}" > "$O/ablate.txt" 2>&1 ;;
    abenv:*)
      # abenv:K=V[;K=V]:KIND:BASES:MINLEN:SHARD -- plan A created under the
      # environment K=V (plan-time switches), B without; same library
      IFS=: read -r _ ENVA KIND BASES MINLEN SHARD <<< "$S"
      AB_ENV_A="${ENVA//;/,}" timeout -k 10 600 python -u tools/ab_interleave.py "$KIND" "$BASES" "$MINLEN" \
        genometools_smax_amd/lib/libgtsmax_hip.so 8 "$SHARD" > "$O/abenv_${KIND}_${ENVA//[=;]/_}_${SHARD//\//of}.txt" 2>&1 ;;
    stamps:*)
      GT_SMAX_LIB=$DIAGLIB timeout -k 10 600 python -u tools/k1_stamps.py "${S#stamps:}" 5 > "$O/stamps_${S#stamps:}.txt" 2>&1 ;;
    rehearse:*)
      # rehearse:W[:BASES] -- bench.py --gpus W as W torchrun ranks on this
      # one GPU, boundary exchange staged through gloo (parity checked)
      IFS=: read -r _ W BASES <<< "$S"
      timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$W" \
        --master-addr 127.0.0.1 --master-port $((29500 + W)) bench.py --gpus "$W" --one-gpu \
        --dist-backend gloo ${BASES:+--bases $BASES} --steps 10 --warmup 2 \
        > "$O/rehearse_w$W.json" 2> "$O/rehearse_w$W.err" ;;
    pmcablate:*)
      # pmcablate:V1,V2,... -- K1 SQ counters under GT_SMAX_DEBUG ablation bits (C3)
      P="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
      for V in $(echo "${S#pmcablate:}" | tr , ' '); do
        (cd /tmp && GT_SMAX_LIB=$DIAGLIB GT_SMAX_DEBUG=$V TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc $P \
          --kernel-include-regex smax_scan -d "$O/pmca_$V" -o p -- python3 "$R/tools/k1_once.py" c3 2 \
          > "$O/pmca_$V.log" 2>&1)
        python3 tools/rocpd_summary.py pmc "$O/pmca_$V.json" smax_scan "c3" "$O/pmca_$V/p_results.db"
        rm -rf "$O/pmca_$V"
      done ;;
    fetchablate:*)
      # fetchablate:V1,V2,... -- K1 FETCH_SIZE under GT_SMAX_DEBUG ablation bits (C3)
      for V in $(echo "${S#fetchablate:}" | tr , ' '); do
        (cd /tmp && GT_SMAX_LIB=$DIAGLIB GT_SMAX_DEBUG=$V TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE \
          --kernel-include-regex smax_scan -d "$O/pmcf_$V" -o p -- python3 "$R/tools/k1_once.py" c3 2 \
          > "$O/pmcf_$V.log" 2>&1)
        python3 tools/rocpd_summary.py pmc "$O/pmcf_$V.json" smax_scan "c3" "$O/pmcf_$V/p_results.db"
        rm -rf "$O/pmcf_$V"
      done ;;
    tilestats:*)
      timeout -k 10 600 python -u tools/tile_stats.py "${S#tilestats:}" > "$O/tilestats_${S#tilestats:}.txt" 2>&1 ;;
    designstats:*)
      # designstats:KIND:BASES:MINLEN -- classification steps per tile by filter / tile size
      IFS=: read -r _ KIND BASES MINLEN <<< "$S"
      timeout -k 10 600 python -u tools/tile_design_stats.py "$KIND" "$BASES" "$MINLEN" \
        > "$O/designstats_${KIND}_$BASES.txt" 2>&1 ;;
    llvstats)
      for C in c3 c5; do
        timeout -k 10 300 python -u tools/llv_window_stats.py $C > "$O/llvstats_$C.txt" 2>&1
      done ;;
    profshards:*)
      W=${S#profshards:}
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/profshards_$W" -o p -- \
        python3 "$R/tools/shard_step.py" human 3e9 20 "$W" > "$O/profshards_$W.txt" 2>&1)
      python3 tools/rocpd_summary.py stats "$O/profshards_$W/p_results.db" "$O/kernel_stats_shards_$W.csv"
      rm -rf "$O/profshards_$W" ;;
    mp:*)
      # mp:CONFIG[:BASES] -- the F2 leg, bench.py --path maxpairs (reference emission order)
      IFS=: read -r _ C BASES <<< "$S"
      timeout -k 10 600 python -u bench.py --path maxpairs --config "$C" ${BASES:+--bases $BASES} \
        > "$O/bench_maxpairs_$C${BASES:+_$BASES}.json" 2> "$O/bench_maxpairs_$C${BASES:+_$BASES}.err" ;;
    mpprof:*)
      # mpprof:CONFIG[:BASES] -- rocprofv3 kernel stats of the F2 leg
      IFS=: read -r _ C BASES <<< "$S"
      T=$C${BASES:+_$BASES}
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/mpprof_$T" -o p -- \
        python3 "$R/bench.py" --path maxpairs --config "$C" ${BASES:+--bases $BASES} --no-cpu-baseline \
        > "$O/mpprof_bench_$T.json" 2> "$O/mpprof_bench_$T.err")
      python3 tools/rocpd_summary.py stats "$O/mpprof_$T/p_results.db" "$O/kernel_stats_maxpairs_$T.csv"
      rm -rf "$O/mpprof_$T" ;;
    mppmc:*|f3pmc:*)
      # mppmc:CONFIG[:BASES] / f3pmc:CONFIG[:BASES] -- HBM bytes per launch of
      # every F2 (mp_*) / F3 (li_*) kernel: --pmc FETCH_SIZE, then WRITE_SIZE
      IFS=: read -r K C BASES <<< "$S"
      T=$C${BASES:+_$BASES}
      if [ "$K" = mppmc ]; then PTH=maxpairs; RX='mp_|rocprim'; else PTH=lcpitv; RX='li_|rocprim'; fi
      for X in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $X --kernel-include-regex "$RX" \
          -d "$O/${K}_${T}_$X" -o p -- python3 "$R/bench.py" --path $PTH --config "$C" ${BASES:+--bases $BASES} \
          --no-cpu-baseline --steps 2 --warmup 1 --prime-s 0 > "$O/${K}_${T}_$X.log" 2>&1)
      done
      python3 tools/rocpd_summary.py pmcall "$O/${K}_$T.json" "$T" "$O/${K}_${T}_FETCH_SIZE/p_results.db" \
        "$O/${K}_${T}_WRITE_SIZE/p_results.db"
      rm -rf "$O/${K}_${T}_FETCH_SIZE" "$O/${K}_${T}_WRITE_SIZE" ;;
    f3sq:*)
      # f3sq:CONFIG[:BASES] -- SQ instruction / wait / LDS counters of every F3 kernel (two passes)
      IFS=: read -r _ C BASES <<< "$S"
      T=$C${BASES:+_$BASES}
      SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
      SQB="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
      for X in A B; do
        if [ $X = A ]; then CS=$SQA; else CS=$SQB; fi
        (cd /tmp && TMPDIR=/tmp timeout -s KILL 300 rocprofv3 --pmc $CS --kernel-include-regex 'li_' \
          -d "$O/f3sq_${T}_$X" -o p -- python3 "$R/bench.py" --path lcpitv --config "$C" ${BASES:+--bases $BASES} \
          --no-cpu-baseline --steps 2 --warmup 1 --prime-s 0 > "$O/f3sq_${T}_$X.log" 2>&1)
      done
      python3 tools/rocpd_summary.py pmcall "$O/f3sq_$T.json" "$T" "$O/f3sq_${T}_A/p_results.db" \
        "$O/f3sq_${T}_B/p_results.db"
      rm -rf "$O/f3sq_${T}_A" "$O/f3sq_${T}_B" ;;
    f3:*)
      # f3:CONFIG[:BASES] -- the F3 leg, bench.py --path lcpitv (intervals + visitor events)
      IFS=: read -r _ C BASES <<< "$S"
      timeout -k 10 600 python -u bench.py --path lcpitv --config "$C" ${BASES:+--bases $BASES} \
        > "$O/bench_lcpitv_$C${BASES:+_$BASES}.json" 2> "$O/bench_lcpitv_$C${BASES:+_$BASES}.err" ;;
    f3prof:*)
      # f3prof:CONFIG[:BASES] -- rocprofv3 kernel stats of the F3 leg
      IFS=: read -r _ C BASES <<< "$S"
      T=$C${BASES:+_$BASES}
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/f3prof_$T" -o p -- \
        python3 "$R/bench.py" --path lcpitv --config "$C" ${BASES:+--bases $BASES} --no-cpu-baseline \
        > "$O/f3prof_bench_$T.json" 2> "$O/f3prof_bench_$T.err")
      python3 tools/rocpd_summary.py stats "$O/f3prof_$T/p_results.db" "$O/kernel_stats_lcpitv_$T.csv"
      rm -rf "$O/f3prof_$T" ;;
    e2ecold:*)
      # cold end-to-end: first call of the drop-in entry point in a fresh process
      timeout -k 10 900 python -u tools/e2e_cold.py "${S#e2ecold:}" 3 > "$O/e2e_cold_${S#e2ecold:}.json" \
        2> "$O/e2e_cold_${S#e2ecold:}.err" ;;
    timeline:*)
      # timeline:SHARD -- kernel trace (CSV) of repeated plan steps of one C3
      # shard: per-kernel durations and the gaps between them
      SH=${S#timeline:}
      (cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv \
        -d "$O/tl_${SH//\//of}" -o p -- python3 "$R/tools/ab_multi.py" human 3e9 20 "$SH" 2 \
        > "$O/tl_${SH//\//of}.log" 2>&1)
      python3 tools/step_timeline.py "$O/tl_${SH//\//of}" > "$O/timeline_${SH//\//of}.txt"
      rm -rf "$O/tl_${SH//\//of}" ;;
    coldprobe)
      # a fresh process's first HIP stream vs the memory the previous one held
      timeout -k 10 600 bash tools/probe/cold_probe.sh "$O/cold_probe.jsonl" > "$O/cold_probe.log" 2>&1 ;;
    e2eshards:*)
      # e2eshards:W -- gt_smax_hip_enumerate_to_buffer(num_gpus=W) on this one
      # device, 3 calls, GT_SMAX_TIMING phases per shard, records vs the oracle
      SHARDS=${S#e2eshards:} CALLS=3 timeout -k 10 600 python -u tools/e2e_breakdown.py 3e9 \
        > "$O/e2e_shards_${S#e2eshards:}.txt" 2>&1 ;;
    e2esweep:*)
      # e2esweep:CONFIG:K=V,..;K=V,.. -- first/second call per runtime setting
      IFS=: read -r _ C SETS <<< "$S"
      IFS=';' read -r -a SA <<< "$SETS"
      timeout -k 10 1000 python -u tools/e2e_cold.py "$C" 2 "${SA[@]}" > "$O/e2e_sweep_$C.json" \
        2> "$O/e2e_sweep_$C.err" ;;
    shards:*)
      W=${S#shards:}
      timeout -k 10 600 python -u tools/shard_step.py human 3e9 20 "$W" > "$O/shards_$W.txt" 2>&1 ;;
    *)
      echo "unknown step $S"; exit 2 ;;
  esac
done
echo "[gpu_round] done $(date +%T)"
