# C4 (B=512 ragged) per-rank scaling emulation with the current kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3n; mkdir -p $O; cd $R
timeout -k 10 600 python tools/scaling_emulation.py > $O/scaling_c4.json 2> $O/scaling_c4.err
echo rc=$?
python -c "
import json; d=json.load(open('$O/scaling_c4.json'))
for n, w in d['worlds'].items(): print(n, w['step_ms'], w['utt_per_s'], w.get('balance'))
print({k: v for k, v in d.items() if k not in ('worlds',)})"
