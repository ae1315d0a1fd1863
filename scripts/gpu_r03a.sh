cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r03a.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu_r03a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03a.log 2>&1 || exit $?
tail -2 gpurun_out/smoke_r03a.log
