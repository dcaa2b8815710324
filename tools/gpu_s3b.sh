set -o pipefail
O=gpurun_out/s3b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surface.py -x -v --timeout 120 --timeout-method thread -k "fill_zero or placement or backward_twice or configs4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2 3 4; do timeout -k 10 200 python bench.py --no-cpu > $O/b$i.json 2>$O/b$i.err || exit 1; python -c "import json;d=json.load(open('$O/b$i.json'));print(d['ms_per_step'],d['kernels'],d['grads_placement'])"; done
