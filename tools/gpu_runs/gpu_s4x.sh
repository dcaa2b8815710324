# the N > 1 bench path on the final code: 2 ranks sharing the box's one GPU (gloo for the host-side collectives)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4x; mkdir -p $O; cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --no-cpu > $O/bench2.json 2> $O/bench2.err
echo rc=$?
cat $O/bench2.json | cut -c1-700
