set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e; mkdir -p $O
ISAL_HIP_ENC_GLDS=8 ISAL_HIP_LOG=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 300 --timeout-method thread -k "test_golden_encode" > $O/pytest_glds8.txt 2>&1
echo rc=$?
grep -v "^  File" $O/pytest_glds8.txt | grep -v "^isal_hip: kernel ec_encode_v16\|route" | head -30
grep "isal_hip: kernel" $O/pytest_glds8.txt | tail -3
