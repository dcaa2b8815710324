# alpha/beta recursion: prefetch depth 16 vs 32 steps, exec-branch vs buffer (out-of-range-dropped) stores; parity first
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4r; mkdir -p $O; cd $R
V='[{"dp_halo":2},{"dp_halo":3},{"dp_halo":4},{"dp_halo":5}]'
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "every_kernel_variant or long_label or alignment" -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --config headline --rounds 7 --variants "$V" > $O/kb_headline.json 2> $O/kb_headline.err && \
timeout -k 10 300 python tools/kbench.py --config ragged64 --rounds 7 --variants "$V" > $O/kb_ragged64.json 2> $O/kb_ragged64.err && \
timeout -k 10 300 python tools/kbench.py --config c2 --rounds 21 --variants "$V" > $O/kb_c2.json 2> $O/kb_c2.err
echo rc=$?
tail -2 $O/parity.log
for f in kb_headline kb_ragged64 kb_c2; do python - <<PY
import json
d=json.load(open("$O/$f.json"))
print("$f")
for v in d.get("variants", d if isinstance(d, list) else []):
    print("  ", json.dumps(v)[:400])
PY
done
