#!/bin/bash
# Round-3 kernel traces: configs[1] graph step with the chase launch (product default) and without (--tune chase=0),
# and the headline line under rocprofv3 --kernel-trace --stats. Output under gpurun_out/tr/.
set -e
O=gpurun_out/tr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_chase -- python3 bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 > $O/c2_chase.json
python3 tools/graph_trace.py $O/c2_chase --last 200 > $O/graph_trace_c2_chase.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_nochase -- python3 bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 --tune chase=0 > $O/c2_nochase.json
python3 tools/graph_trace.py $O/c2_nochase --last 200 > $O/graph_trace_c2_nochase.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/headline -- python3 bench.py --config headline --steps 10 --warmup 3 > $O/headline.json
echo done
