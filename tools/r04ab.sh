# Round-4 A/B on one MI355X: optional GPU test subset ($TESTS), then the plain bench (HIP-event roofline, no
# profiler) for the default settings and for each AB_ENVS variant (space-separated VAR=value), $REPS times each,
# alternating, so box drift hits every variant alike.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab4_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/ab4_tests.log; exit 1; }
  tail -1 gpurun_out/ab4_tests.log
fi
run() {  # $1 tag, rest: env settings
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-300} --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary $BENCH_EXTRA > gpurun_out/ab4_$tag.json 2> gpurun_out/ab4_$tag.err || { echo BENCHFAIL $tag; tail gpurun_out/ab4_$tag.err; exit 1; }
  python - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab4_{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "it/s %.1f ms/it %.4f k1 %.2f us frac %.3f cold %s" % (d["value"], d["ms_per_step"], 1e3 * r["k1_avg_ms"], r["frac"],
      round(r["cold_cache"]["frac"], 3) if "cold_cache" in r else None),
      {k: round(v * 1e3, 1) for k, v in d["kernel_ms"].items()})
PY
}
for rep in $(seq ${REPS:-1}); do
  run A$rep || exit 1
  k=0
  # a variant may set several variables, comma-separated (VAR1=a,VAR2=b)
  for kv in $AB_ENVS; do k=$((k+1)); run B${k}_$rep $(echo "$kv" | tr ',' ' ') || exit 1; done
done
