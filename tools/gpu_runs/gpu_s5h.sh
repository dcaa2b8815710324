# fused joint sweeps through its launch variants: 3 W-chunk buffers, frame-by-frame / row-parallel d_enc,d_pred reduce
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s5h; mkdir -p $O; cd $R
run() { tag=$1; shift; env "$@" timeout -k 10 600 python -u -m pytest tests/test_gpu_joint.py -k test_joint_random_cases -q --timeout 300 --timeout-method thread > $O/$tag.log 2>&1; echo "$tag rc=$? $(tail -1 $O/$tag.log)"; }
run nbuf3 MRNNT_FUZZ_TUNE=joint_nbuf=3 MRNNT_FUZZ_FIRST=2000 MRNNT_JOINT_CASES=200
run reduce_frames MRNNT_FUZZ_TUNE=joint_reduce_sparse=1 MRNNT_FUZZ_FIRST=3000 MRNNT_JOINT_CASES=200
run reduce_rows MRNNT_FUZZ_TUNE=joint_reduce_sparse=2 MRNNT_JOINT_BIG=1 MRNNT_FUZZ_FIRST=4000 MRNNT_JOINT_CASES=100
