cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/polish_prof.py 10000 1 5 20 > gpurun_out/polprof.log 2>&1; rc=$?; tail -8 gpurun_out/polprof.log; exit $rc
