#!/bin/bash
# The one GPU-box runner (replaces round 4's one-off tools/r04_*.sh).  Every step runs under its own
# time limit; the first failing step ends the call (no retries, nothing more on the GPU).
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]        (from the repo root, via gpurun)
#
# Output goes to gpurun_out/TAG/.  Steps:
#   tests[=PYTEST_K]   pytest -m gpu (optionally -k PYTEST_K)          -> gpu_tests.log
#   smoke              __graft_entry__.smoke()                         -> smoke.log
#   bench[=ARGS]       bench.py --steps 20 --warmup 5 ARGS             -> bench_<n>.json (n = step index)
#   c4[=ARGS]          bench.py --config C4 ARGS                       -> bench_c4_<n>.json
#   prof_kv            rocprofv3 --kernel-trace --stats over the C2 headline + tools/roofline_rocprof.py
#   prof[=ARGS]        rocprofv3 --kernel-trace --stats over bench.py ARGS -> prof_<n>/
#   pmc[=REGEX]        tools/gpu_pmc.sh passes (PMC only with --kernel-trace)
#   configs=LIST       tools/bench_configs.py --only LIST              -> configs_<n>.jsonl
#   latency[=ARGS]     tools/latency_probe.py ARGS                     -> latency_<n>.jsonl
#   py=SCRIPT[:ARGS]   python3 SCRIPT ARGS (any probe under tools/)    -> py_<n>.log
#   bin=EXE[:ARGS]     a probe binary built here (e.g. tools/sha_lone)  -> bin_<n>.log
# Environment: NWCRYPTO_LIB=path selects a variant library (A/B runs, tools/build_variants.sh);
# STEP_TIMEOUT overrides the per-step limit (seconds).
set -o pipefail
TAG=${1:?usage: gpu_run.sh TAG STEP [STEP ...]}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0

die() { echo "STEP $n ($1) FAILED"; [ -f "$2" ] && tail -25 "$2"; exit 1; }
lim() { echo "${STEP_TIMEOUT:-$1}"; }
summ() {   # one-line summary of a bench JSON line
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(d["config"]["workload"][:60], "| %.1f M sigs/s | %.3f ms/step | k_verify %.4f ms frac %.3f"
      % (d["value"] / 1e6, d["ms_per_step"], r.get("avg_launch_ms", float("nan")), r.get("frac", float("nan"))))
EOF
}

for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "== step $n: $step"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 "$(lim 1100)" python -u -m pytest tests -m gpu -x -v --durations=20 --timeout 300 \
        --timeout-method thread "${K[@]}" > "$OUT/gpu_tests.log" 2>&1 || die tests "$OUT/gpu_tests.log"
      tail -3 "$OUT/gpu_tests.log" ;;
    smoke)
      timeout -k 10 "$(lim 300)" python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || die smoke "$OUT/smoke.log"
      cat "$OUT/smoke.log" ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 600)" python3 -u bench.py --steps 20 --warmup 5 $arg > "$OUT/bench_$n.json" \
        2> "$OUT/bench_$n.err" || die bench "$OUT/bench_$n.err"
      summ "$OUT/bench_$n.json" ;;
    c4)
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 900)" python3 -u bench.py --config C4 --steps 10 --warmup 2 $arg > "$OUT/bench_c4_$n.json" \
        2> "$OUT/bench_c4_$n.err" || die c4 "$OUT/bench_c4_$n.err"
      summ "$OUT/bench_c4_$n.json" ;;
    prof_kv)
      timeout -k 10 "$(lim 400)" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_kv" -o kv -- \
        python3 bench.py --steps 10 --warmup 2 --c4-steps 0 --no-cpu-baseline --latency-samples 0 --no-extras --digest-batches 0 \
        > "$OUT/bench_kv.json" 2> "$OUT/prof_kv.log" || die prof_kv "$OUT/prof_kv.log"
      python3 tools/roofline_rocprof.py "$OUT/prof_kv/kv_kernel_trace.csv" --bench "$OUT/bench_kv.json" --skip 2 \
        --take 10 > "$OUT/roofline_rocprof.json" && cat "$OUT/roofline_rocprof.json"
      cut -d, -f1-4 "$OUT/prof_kv/kv_kernel_stats.csv" | cut -c1-150 | head -14 ;;
    prof)
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 600)" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$n" -o p -- \
        python3 bench.py --no-cpu-baseline --latency-samples 0 $arg > "$OUT/prof_$n.json" 2> "$OUT/prof_$n.log" \
        || die prof "$OUT/prof_$n.log"
      cut -d, -f1-4 "$OUT/prof_$n/p_kernel_stats.csv" | cut -c1-150 | head -20 ;;
    pmc)
      timeout -k 10 "$(lim 900)" bash tools/gpu_pmc.sh "$TAG/pmc_$n" "${arg:-k_verify|k_finish|k_sha512}" \
        > "$OUT/pmc_$n.log" 2>&1 || die pmc "$OUT/pmc_$n.log"
      tail -3 "$OUT/pmc_$n.log" ;;
    configs)
      timeout -k 10 "$(lim 900)" python3 -u tools/bench_configs.py --only "${arg:?configs=LIST}" --cpu-seconds 0 \
        > "$OUT/configs_$n.jsonl" 2> "$OUT/configs_$n.err" || die configs "$OUT/configs_$n.err"
      cut -c1-300 "$OUT/configs_$n.jsonl" ;;
    latency)
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 400)" python3 -u tools/latency_probe.py $arg > "$OUT/latency_$n.jsonl" \
        2> "$OUT/latency_$n.err" || die latency "$OUT/latency_$n.err"
      cut -c1-300 "$OUT/latency_$n.jsonl" ;;
    py)
      s=${arg%%:*}; a=""; [ "$s" != "$arg" ] && a=${arg#*:}
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 600)" python3 -u "$s" $a > "$OUT/py_$n.log" 2>&1 || die py "$OUT/py_$n.log"
      tail -20 "$OUT/py_$n.log" | cut -c1-400 ;;
    bin)
      s=${arg%%:*}; a=""; [ "$s" != "$arg" ] && a=${arg#*:}
      # shellcheck disable=SC2086
      timeout -k 10 "$(lim 300)" "./$s" $a > "$OUT/bin_$n.log" 2>&1 || die bin "$OUT/bin_$n.log"
      tail -20 "$OUT/bin_$n.log" | cut -c1-400 ;;
    *)
      echo "unknown step: $step"; exit 2 ;;
  esac
done
exit 0
