set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d; mkdir -p $O
# parity of the LDS-DMA staged wide encode first: one device-resident test, then the rest
ISAL_HIP_ENC_GLDS=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "test_encode_load_groups_vs_oracle" > $O/pytest_glds8_first.txt 2>&1 || { echo PYTEST FAIL; grep -v "^  File" $O/pytest_glds8_first.txt | tail -30; exit 1; }
tail -2 $O/pytest_glds8_first.txt
ISAL_HIP_ENC_GLDS=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "load_groups or xor_fast_path or maximum_stripe or random_shapes or golden_encode" > $O/pytest_glds8.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_glds8.txt; exit 1; }
tail -2 $O/pytest_glds8.txt
ISAL_HIP_ENC_GLDS=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "load_groups or xor_fast_path" > $O/pytest_glds4.txt 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_glds4.txt; exit 1; }
tail -2 $O/pytest_glds4.txt
for r in 1 2; do
 for shape in "20 6 4194304 64" "20 8 4194304 64" "10 8 1048576 1024" "10 6 1048576 1024"; do
  set -- $shape
  for g in 0 4 6 8; do
    ISAL_HIP_ENC_GLDS=$g timeout -k 10 300 python bench.py --k $1 --p $2 --len $3 --stripes $4 --no-cpu-baseline > $O/b.json 2>$O/b.err || { echo BENCH FAIL; tail $O/b.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$O/b.json')); r=d['roofline']
print(json.dumps({'round':$r,'k':$1,'p':$2,'glds':$g,'frac':r['frac'],'launch_ms':r['launch_ms'],'kernel':r['kernel'],'self_check':d['self_check'],'copy':r.get('copy_ceiling',{}).get('gb_s')}))" >> $O/ab.jsonl
  done
 done
done
cat $O/ab.jsonl
