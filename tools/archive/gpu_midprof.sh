cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u tools/mid_polish_prof.py 10000 100 2 3 > gpurun_out/midprof.log 2>&1; rc=$?; tail -5 gpurun_out/midprof.log; exit $rc
