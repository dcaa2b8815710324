# per-step forward/backward times over 60 steps in two processes (time-dependent slowdown of the gradient kernel?)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3g; mkdir -p $O; cd $R
timeout -k 10 300 python tools/step_trace.py --steps 60 > $O/trace1.jsonl 2> $O/trace1.err && \
timeout -k 10 300 python tools/step_trace.py --steps 60 > $O/trace2.jsonl 2> $O/trace2.err
echo rc=$?
for i in 1 2; do python -c "
import json; L=[json.loads(l) for l in open('$O/trace$i.jsonl')]
print('proc $i bwd:', ' '.join('%.1f' % d['bwd_ms'] for d in L))
print('proc $i fwd:', ' '.join('%.1f' % d['fwd_ms'] for d in L))"; done
