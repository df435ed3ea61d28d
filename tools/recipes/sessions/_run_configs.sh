cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py > gpurun_out/configs.log 2>&1
echo rc=$?
tail -15 gpurun_out/configs.log
