#!/bin/bash
# One parametrised GPU job (replaces the per-experiment gpu_rNN*.sh wrappers).
#   bash scripts/gpu_job.sh TAG STEP [STEP ...]
# Every step runs under its own time limit and writes gpurun_out/TAG/<step>.log;
# the job stops at the first failing step (no GPU step runs after a failure).
# Steps:
#   pytest      the GPU test suite (one process)
#   smoke       __graft_entry__.smoke()
#   b20 / b100  bench.py at the driver setting (20 steps, 5 warm-up) / 100 steps, no components
#   b20nk       the same 20 steps without per-kernel HIP events in the timed steps
#   bench       bench.py with every component and the CPU baseline (the round-end line)
#   bench20     the same at the driver setting (20 steps, 5 warm-up)
#   pmccopy     this job's prof summary into profiles/ (so the bench lines after it cite it)
#   tl20        tuning build, 20 steps, LDSP_PROF_TIMELINE dump + scripts/prof_timeline.py
#   chains      scripts/chains_bench.py
#   channels    scripts/channels_run.py (8 AMRadio chains on one GPU)
#   c3spread    config-3 launch spread study (scripts/c3_spread.py)
#   iirpmc      scripts/iir_pmc.sh (k_iir_modal kernel stats, HBM bytes, SQ / VALU-type counters)
#   c3ab        config 3 (firbench) with build_ab/ (the previous build) and the product, twice, alternating
#   ab:<file>:<pkg>,<pkg>..  a script with each package build in turn (LDSP_PKG_DIR), twice
#   sqab:<pkg>,..  SQ issue counters of k_iir_modal per package build (scripts/iir_sq_ab.sh)
#   ubench:<b>  a prebuilt microbenchmark scripts/ubench/<b>
#   p20:<pkg>   bench.py at the driver setting on the package build in <pkg> (A/B builds)
#   pb:<pkg>    scripts/batched_run.py on the package build in <pkg>
#   tb:K=V,...  bench.py at the driver setting with components (no CPU baseline) on the tuning build
#   prof        rocprofv3 kernel stats + PMC passes (scripts/prof_round.sh TAG)
#   py:<file>   python <file> (a one-off script under scripts/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=$1; shift
o=gpurun_out/$tag
mkdir -p "$o"
export TMPDIR=/tmp
B="python -u bench.py --no-cpu-baseline --no-components"
run() {   # step name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$o/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  grep -E '^\{|passed|failed|error|smoke ok' "$o/$name.log" | tail -3 | cut -c1-400
  [ $rc -eq 0 ] || { tail -15 "$o/$name.log"; exit $rc; }
}
for step in "$@"; do
  case $step in
    pytest) run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytest:*) k=${step#pytest:}; run "pytest_$k" 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$k" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    b20) run b20 400 $B --steps 20 --warmup 5 ;;
    b20nk) run b20nk 400 $B --steps 20 --warmup 5 --no-kprof ;;
    b100) run b100 400 $B --steps 100 ;;
    bench) run bench 900 python -u bench.py ;;
    bench20) run bench20 900 python -u bench.py --steps 20 --warmup 5 ;;
    pmccopy) cp "gpurun_out/prof/$tag/summary.json" "profiles/${tag}_pmc_summary.json" && echo "[pmccopy] profiles/${tag}_pmc_summary.json" ;;
    tl20|tl20:*) kv=${step#tl20}; kv=${kv#:}; name="tl20$(echo "_$kv" | tr ',=' '_-')"; rm -f "$o/$name.txt"
          env $(echo "$kv" | tr ',' ' ') LDSP_PKG_DIR=build_tuning LDSP_PROF_TIMELINE="$o/$name.txt" \
            timeout -k 10 400 $B --steps 20 --warmup 5 --no-kprof > "$o/$name.log" 2>&1
          rc=$?; echo "[$name] rc=$rc"; grep '^{' "$o/$name.log" | cut -c1-330; [ $rc -eq 0 ] || exit $rc
          python scripts/prof_timeline.py "$o/$name.txt" > "$o/${name}_summary.txt" 2>&1; head -3 "$o/${name}_summary.txt"; tail -1 "$o/${name}_summary.txt" ;;
    chains) run chains 400 python -u scripts/chains_bench.py ;;
    channels) run channels 400 python -u scripts/channels_run.py ;;
    c3spread) FIRBENCH_REPS=16 PMC_OUT="$o/c3" run c3pmc 600 bash scripts/fir_c3_pmc.sh
              python scripts/c3_spread.py "$o/c3" > "$o/c3_spread.json"; head -c 1500 "$o/c3_spread.json"; echo ;;
    iirpmc) IIRPMC_OUT="$o/iirpmc" run iirpmc 900 bash scripts/iir_pmc.sh
            python scripts/pmc_kernel.py "$o/iirpmc" > "$o/iirpmc_summary.json"; head -c 2500 "$o/iirpmc_summary.json"; echo ;;
    c3ab) for pk in build_ab python-liquiddsp_amd build_ab python-liquiddsp_amd; do
            FIRBENCH_N=1048576 FIRBENCH_TAPS=255 FIRBENCH_REPS=12 LDSP_PKG_DIR=$pk run "c3_$(basename $pk)" 300 python -u scripts/firbench.py
          done ;;
    ab:*) spec=${step#ab:}; f=${spec%%:*}; pkgs=${spec#*:}
          for rep in 1 2; do for pk in $(echo "$pkgs" | tr ',' ' '); do
            LDSP_PKG_DIR=$pk run "ab_$(basename "$f" .py)_$(basename "$pk")_$rep" 300 python -u "$f"
          done; done ;;
    sqab:*) pk=${step#sqab:}; run sqab 600 bash scripts/iir_sq_ab.sh "$o/sqab" $(echo "$pk" | tr ',' ' '); cat "$o/sqab.log" | grep -v '^$' | tail -8 ;;
    ubench:*) f=${step#ubench:}; run "ub_$f" 120 "scripts/ubench/$f" ;;
    prof) run prof 1100 bash scripts/prof_round.sh "$tag" ;;
    py:*) f=${step#py:}; run "$(basename "$f" .py)" 600 python -u "$f" ;;
    tpy:*) f=${step#tpy:}; kv=""; case $f in *:*) kv=${f#*:}; f=${f%%:*};; esac
           name="t_$(basename "$f" .py)$(echo "${kv:+_$kv}" | tr ',=' '_-')"
           env $(echo "$kv" | tr ',' ' ') LDSP_PKG_DIR=build_tuning timeout -k 10 600 python -u "$f" > "$o/$name.log" 2>&1
           rc=$?; echo "[$name] rc=$rc"; grep '^{' "$o/$name.log" | cut -c1-400; [ $rc -eq 0 ] || { tail -15 "$o/$name.log"; exit $rc; } ;;
    t20:*) kv=${step#t20:}; name="t20_$(echo "$kv" | tr ',=' '_-')"
           env $(echo "$kv" | tr ',' ' ') LDSP_PKG_DIR=build_tuning \
             timeout -k 10 400 $B --steps 20 --warmup 5 > "$o/$name.log" 2>&1
           rc=$?; echo "[$name] rc=$rc"; grep '^{' "$o/$name.log" | cut -c1-330
           grep -o '"single_stream_ms_per_step": [0-9.]*\|"k_pll_cand": {[^}]*}\|"k_agc_chunks": {[^}]*}\|"k_agc_runfix": {[^}]*}\|"k_pll_walk": {[^}]*}\|"repairs": [0-9]*' "$o/$name.log" | tr '\n' ' '; echo
           [ $rc -eq 0 ] || { tail -15 "$o/$name.log"; exit $rc; } ;;
    p20:*) pk=${step#p20:}; name="p20_$(basename "$pk")"
           LDSP_PKG_DIR=$pk timeout -k 10 400 $B --steps 20 --warmup 5 > "$o/$name.log" 2>&1
           rc=$?; echo "[$name] rc=$rc"; grep '^{' "$o/$name.log" | cut -c1-330
           grep -o '"single_stream_ms_per_step": [0-9.]*\|"k_agc_chunks": {[^}]*}\|"k_agc_runfix": {[^}]*}\|"k_pll_cand": {[^}]*}' "$o/$name.log" | tr '\n' ' '; echo
           [ $rc -eq 0 ] || { tail -15 "$o/$name.log"; exit $rc; } ;;
    tb:*) kv=${step#tb:}; name="tb_$(echo "$kv" | tr ',=' '_-')"
          env $(echo "$kv" | tr ',' ' ') LDSP_PKG_DIR=${TB_PKG:-build_tuning} timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$o/$name.log" 2>&1
          rc=$?; echo "[$name] rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"channels_per_gpu[a-z_0-9]*": {[^}]*}' "$o/$name.log" | cut -c1-200
          [ $rc -eq 0 ] || { tail -15 "$o/$name.log"; exit $rc; } ;;
    pb:*) pk=${step#pb:}; LDSP_PKG_DIR=$pk run "pb_$(basename "$pk")" 300 python -u scripts/batched_run.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
