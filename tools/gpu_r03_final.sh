#!/bin/bash
# Round-3 final profile set (profiles/r03): GPU tests, smoke, the driver's bench command, rocprofv3
# kernel stats of C2 / C3 / C5 / the JPEG stage, PMC passes + HBM traffic for C2 / C3 / C5 (as
# tools/gpu_r03_profiles.sh without the LDS-conflict attribution passes, which need ablation builds).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/r03; export TMPDIR=/tmp
O="$R/gpurun_out/r03"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
echo "bench ok"
cd /tmp
prof() { # name, program...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n" -o run --output-format csv -- "$@" > "$O/prof_$n.log" 2>&1 || { tail -5 "$O/prof_$n.log"; return 1; }
  cp "$O/prof_$n/run_kernel_stats.csv" "$O/${n}_kernel_stats.csv"
}
prof c2 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extra || exit 1
prof c3 python3 "$R/tools/kbench.py" C3 default || exit 1
prof c5 python3 "$R/tools/c5_run.py" 30 || exit 1
prof jpeg python3 "$R/tools/jpeg_ab.py" || exit 1
echo "rocprof ok"
cd "$R"
for cfg in C2 C3 C5; do
  tools/gpu_pmc.sh $cfg > $O/pmc_$cfg.txt 2>&1 || { echo "pmc $cfg failed"; tail $O/pmc_$cfg.txt; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc/$cfg $cfg $O/traffic_r03.json > $O/pmc_${cfg}_summary.txt || exit 1
done
echo "pmc ok"
cd /tmp
echo "all ok"
