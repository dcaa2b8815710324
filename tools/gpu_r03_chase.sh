#!/bin/bash
# Round-3 chase measurements (configs[1] HIP-graph step, headline): chase on (product default) vs off (dev build,
# --tune chase=0), plus rocprofv3 kernel traces of the c2 graph step. Output under gpurun_out/chase/.
set -e
O=gpurun_out/chase
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { timeout -k 10 300 python -u bench.py --no-cpu "$@"; }
run --config c2 --graph --steps 300 --warmup 30 > $O/c2_graph_chase_1.json
run --config c2 --graph --steps 300 --warmup 30 --tune chase=0 > $O/c2_graph_nochase_1.json
run --config c2 --graph --steps 300 --warmup 30 > $O/c2_graph_chase_2.json
run --config c2 --graph --steps 300 --warmup 30 --tune chase=0 > $O/c2_graph_nochase_2.json
run --config c2 --graph --steps 300 --warmup 30 --tune chase=1 --tune chase_depth=8 > $O/c2_graph_chase_d8.json
run --config headline --steps 10 --warmup 3 > $O/headline_chase.json
run --config headline --steps 10 --warmup 3 --tune chase=0 > $O/headline_nochase.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c2_chase -- python3 bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 > $O/trace_c2_chase.json
python3 tools/graph_trace.py $O/trace_c2_chase --last 200 > $O/graph_trace_c2_chase.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c2_nochase -- python3 bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 --tune chase=0 > $O/trace_c2_nochase.json
python3 tools/graph_trace.py $O/trace_c2_nochase --last 200 > $O/graph_trace_c2_nochase.json
find $O -name "*_stats.csv" -o -name "*kernel_trace.csv" | head -20
echo done
