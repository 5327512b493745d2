cd $GRAFT_REPO_ROOT
export AMD_SERIALIZE_KERNEL=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "doc_farmer or test_farmer_ph_matches_oracle" > gpurun_out/t1.log 2>&1; rc=$?; tail -30 gpurun_out/t1.log; exit $rc
