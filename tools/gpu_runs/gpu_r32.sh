# A/B of the joint epilogue: packed f32 (v_pk_*) vs scalar vs scalar epilogue + packed tanh build; bench box-copy probe
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r32; mkdir -p $O; cd $R
for v in packed scalar mixed packed scalar mixed; do
  MRNNT_LIB=$R/ab/$v/libmonotonic_rnnt_amd.so timeout -k 10 240 python tools/joint_bench.py --no-unfused --steps 5 >> $O/joint_$v.json 2>> $O/err.log || exit 1
done
MRNNT_LIB=$R/ab/mixed/libmonotonic_rnnt_amd.so timeout -k 10 240 python tools/joint_bench.py --no-unfused --H 256 --steps 5 >> $O/joint_mixed_h256.json 2>> $O/err.log &&
MRNNT_LIB=$R/ab/packed/libmonotonic_rnnt_amd.so timeout -k 10 240 python tools/joint_bench.py --no-unfused --H 256 --steps 5 >> $O/joint_packed_h256.json 2>> $O/err.log &&
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2>> $O/err.log
echo rc=$?
for f in $O/*.json; do echo "== $f"; python -c "
import json,sys
for l in open('$f'):
    d=json.loads(l)
    if 'fused' in d: print(d['fused']['kernels_ms'], d['fused']['ms_per_step'])
    else: print(d['value'], d['roofline'])
"; done
