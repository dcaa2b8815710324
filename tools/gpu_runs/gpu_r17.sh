set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r17
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 3 --warmup 1 > $O/jb.json 2> $O/jb.err
echo rc=$?
