# joint pipelined variants: NW 8/4, ds_read ring 2/4; PMC of the pipelined kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r34; mkdir -p $O; cd $R
run() { # label lib tune...
  local lab=$1 lib=$2; shift 2
  local args=""; for t in "$@"; do args="$args --tune $t"; done
  MRNNT_LIB=$lib timeout -k 10 240 python tools/joint_bench.py --no-unfused --steps 5 $args | sed "s/^/$lab /" >> $O/ab.txt 2>> $O/err.log
}
D=$R/monotonic-rnnt_amd/libmonotonic_rnnt_amd.so; G=$R/ab/ring4/libmonotonic_rnnt_amd.so
for rep in 1 2; do
  run plain $D joint_pipe=0 && run pipe_nw8 $D joint_pipe=1 && run pipe_nw4 $D joint_pipe=1 joint_nw=4 && \
  run ring4_nw8 $G joint_pipe=1 && run ring4_nw4 $G joint_pipe=1 joint_nw=4 || exit 1
done
cd /tmp && export TMPDIR=/tmp
MRNNT_TUNE=joint_pipe=1 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 1 --warmup 1 > $O/p1.json 2> $O/p1.err && \
MRNNT_TUNE=joint_pipe=1 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU -d $O/p2 -o run --output-format csv -- python3 $R/tools/joint_bench.py --no-unfused --steps 1 --warmup 1 > $O/p2.json 2> $O/p2.err
echo rc=$?
python3 $R/tools/pmc_kernel.py $O/p1 $O/p2 --match joint_fwd --match joint_bwd
python3 - <<'PY'
import json
for l in open('/root/repo/gpurun_out/r34/ab.txt'):
    lab, js = l.split(' ', 1); d = json.loads(js)
    print(f"{lab:10s}", d['fused']['kernels_ms'], d['fused']['ms_per_step'])
PY
