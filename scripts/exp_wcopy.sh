# k_ba_wcopy experiment: byte-array parity subset, then the C4 bench (kernel times)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -k "byte_array or plain_chain or fuzz or c4 or pyarrow or all_types" > gpurun_out/t_wcopy.log 2>&1; rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/t_wcopy.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu --no-e2e > gpurun_out/b_c4.log 2>&1 || exit 1
python - <<'P'
import json
l=[x for x in open("gpurun_out/b_c4.log") if x.startswith('{')][-1]; d=json.loads(l)
print(d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_ms'] for k,v in d['kernels'].items() if v['avg_ms']>0.02})
P
