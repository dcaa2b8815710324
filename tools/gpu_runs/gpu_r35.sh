# s_memtime phase split of the pipelined joint forward kernel (diagnostic build ab/stamp)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r35; mkdir -p $O; cd $R
for H in 512 256; do
  MRNNT_LIB=$R/ab/stamp/libmonotonic_rnnt_amd.so MRNNT_TUNE=joint_pipe=1 timeout -k 10 240 python tools/joint_stamps.py --H $H >> $O/stamps.json 2>> $O/err.log || exit 1
done
cat $O/stamps.json
