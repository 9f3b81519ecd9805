cd "$GRAFT_REPO_ROOT" && timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; exit $rc
