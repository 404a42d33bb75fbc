#!/bin/bash
# Round-6 closing profile set (profiles/r06f): GPU tests, smoke, the driver's bench command, rocprofv3 kernel
# stats of the C2 contract run, C3 (one-launch record kernel), C5, the JPEG stage and the C2 workload
# with CUBIC / AREA / LANCZOS4, then PMC passes + HBM traffic for C2 / C3 / C5 and the three resize methods.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/r06f; export TMPDIR=/tmp
O="$R/gpurun_out/r06f"
if [ -n "$PMC_ONLY" ]; then SKIP_TESTS=1; fi
if [ -z "$PMC_ONLY" ]; then
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
fi
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python tools/summarize_bench.py $O/bench.json
cd /tmp
prof() { # name, program...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run --output-format csv -- "$@" > "$O/prof_$n.log" 2>&1 || { tail -5 "$O/prof_$n.log"; return 1; }
  cp "$O/prof_$n/run_kernel_stats.csv" "$O/${n}_kernel_stats.csv"
}
prof c2 python3 "$R/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --no-extra || exit 1
prof c3 python3 "$R/tools/kbench.py" C3 default || exit 1
prof c5 python3 "$R/tools/c5_run.py" 30 || exit 1
prof jpeg python3 "$R/tools/jpeg_stage.py" gpu || exit 1
for m in CUBIC AREA LANCZOS4; do prof c2_$m python3 "$R/tools/kbench.py" C2:$m default || exit 1; done
echo "rocprof ok"
cd "$R"
timeout -k 10 300 python3 -u tools/interp_steps.py 20 > $O/interp_steps.txt 2>&1 || exit 1
for m in 1 0; do AEON_HIP_JPEG_COPY_STREAM=$m timeout -k 10 200 python3 -u tools/jpeg_stage.py gpu > $O/jpeg_stage_copy$m.json 2>/dev/null || exit 1; done
bash tools/c5_ab.sh pair > $O/c5_steps.txt 2>&1 || exit 1
fi
cd "$R"
[ -n "$SKIP_PMC" ] && exit 0
for cfg in C2 C3 C5 C2:CUBIC C2:AREA C2:LANCZOS4; do
  tools/gpu_pmc.sh $cfg > $O/pmc_$cfg.txt 2>&1 || { echo "pmc $cfg failed"; tail $O/pmc_$cfg.txt; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc/$cfg $cfg $O/traffic_r06f.json > $O/pmc_${cfg}_summary.txt || exit 1
done
echo "pmc ok"
