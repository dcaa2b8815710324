# fuzz failures (seeds 133, 134, 157: infinite cost of utterance 0) after zeroing the lp pads:
# the poisoned-workspace regression test, the failing sequence, then the whole sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s4j; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k stale_workspace -v --timeout 120 --timeout-method thread > $O/stale.log 2>&1 && \
timeout -k 10 120 python -u tools/debug/fuzz_repro.py 131,132,133,134 > $O/repro.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/stale.log | tail -8
grep -v Warning $O/repro.log | tail -12
tail -n 5 $O/fuzz.log
