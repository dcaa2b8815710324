#!/bin/bash
# Round-3 measurements after the interleaved lp layout: chase probes, configs[1] graph step chase on/off, headline,
# fused-joint 8- vs 4-wave workgroups. Output under gpurun_out/m2/.
set -e
O=gpurun_out/m2
mkdir -p $O
timeout -k 10 200 python -u tools/kbench.py --config c2 --rounds 40 --variants "$(cat tools/chase_variants.json)" > $O/kbench_c2.json 2> $O/kbench_c2.err
timeout -k 10 300 python -u bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 > $O/c2_graph_chase.json
timeout -k 10 300 python -u bench.py --no-cpu --config c2 --graph --steps 300 --warmup 30 --tune chase=0 > $O/c2_graph_nochase.json
timeout -k 10 300 python -u bench.py --no-cpu --config headline --steps 10 --warmup 3 > $O/headline.json
timeout -k 10 400 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 > $O/joint_h512_nw8.json
timeout -k 10 400 python -u tools/joint_bench.py --no-unfused --steps 5 --warmup 2 --tune joint_nw=4 > $O/joint_h512_nw4.json
echo done
