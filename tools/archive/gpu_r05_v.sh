cd $GRAFT_REPO_ROOT && PHGPU_VERBOSE=1 timeout -k 10 120 python tools/fin_prof.py 10000 5 2>&1 | grep -E "phgpu|pass" | head -8
