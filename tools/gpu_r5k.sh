# Final GPU test pass of the committed tree: pytest -m gpu then smoke(), logs into gpurun_out/r5k/.
set -e
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
