# log-softmax with packed fp32 fma/add (new) vs scalar (tools/debug/libold.so), f32 and bf16, alternating processes
# parity of the new build, then alternating bench processes at f32 and bf16
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4h; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --acts-dtype bf16 > $O/new_bf_$i.json 2> $O/e1 && \
  MRNNT_LIB=$R/tools/debug/libold.so timeout -k 10 200 python bench.py --no-cpu --acts-dtype bf16 > $O/old_bf_$i.json 2> $O/e2 && \
  timeout -k 10 200 python bench.py --no-cpu > $O/new_f32_$i.json 2> $O/e3 && \
  MRNNT_LIB=$R/tools/debug/libold.so timeout -k 10 200 python bench.py --no-cpu > $O/old_f32_$i.json 2> $O/e4 || break
done
echo rc=$?
tail -n 1 $O/pytest.log
for f in new_bf_1 old_bf_1 new_bf_2 old_bf_2 new_f32_1 old_f32_1 new_f32_2 old_f32_2; do python -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['kernels']['log_softmax'])"; done
