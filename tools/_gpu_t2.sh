set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/lib_digest.py > gpurun_out/t2_digest_new.txt 2>&1 || exit 1
STF_LIB=$GRAFT_REPO_ROOT/abbase/libstfunet_hip.so timeout -k 10 200 python tools/lib_digest.py > gpurun_out/t2_digest_base.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2_tests.log 2>&1 || { tail -30 gpurun_out/t2_tests.log; exit 1; }
bash tools/ab_lib.sh 1 > gpurun_out/t2_ab.txt 2>&1
