set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1c
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rs > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
echo rc=$?
tail -n 3 $O/pytest.log
cat $O/bench.json $O/bench_2rank_gloo.json
