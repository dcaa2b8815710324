set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r31
mkdir -p $O
cd $R
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err
echo rc=$?
cat $O/bench_2rank_gloo.json
tail -n 5 $O/bench_2rank_gloo.err
