set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_sg.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu --pods3 2000 --force-shard > gpurun_out/c3s_g.json 2> gpurun_out/c3s_g.err || exit $?
KSIM_NO_SHARD_GRAPH=1 timeout -k 10 300 python3 -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu --pods3 2000 --force-shard > gpurun_out/c3s_ng.json 2> gpurun_out/c3s_ng.err
