set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06p
timeout -k 10 300 python3 -u tools/r06_tbclk.py > gpurun_out/r06p/tbclk.txt 2>&1 || exit $?
cat gpurun_out/r06p/tbclk.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06p/prof -o c3 --output-format csv -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu > gpurun_out/r06p/bench_c3.json 2> gpurun_out/r06p/bench_c3.err || exit $?
find gpurun_out/r06p/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06p/pytest.txt 2>&1; tail -3 gpurun_out/r06p/pytest.txt
