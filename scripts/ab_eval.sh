cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-station --no-cpu-baseline > gpurun_out/bench_fused.log 2>&1 && \
LOMPC_FUSED=0 timeout -k 10 300 python bench.py --no-station --no-cpu-baseline > gpurun_out/bench_unfused.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-station > gpurun_out/prof.log 2>&1
