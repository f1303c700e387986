# which round-4 switch breaks test_unet_forward_backward_vs_reference[fp32_x6]: one pytest per
# setting (each under its own timeout; a failing setting does not stop the others)
set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T='tests/test_gpu_parity.py::test_unet_forward_backward_vs_reference tests/test_gpu_parity.py::test_unet_unit_gain_fwd_bwd_vs_fp64'
for v in def sk0 hb0 wg0 all0; do
  case $v in def) ev="";; sk0) ev="DN_X6_SPLITK=0";; hb0) ev="DN_X6_HEAD_BWD=0";; wg0) ev="DN_X6_WGRAD1=0";; all0) ev="DN_X6_SPLITK=0 DN_X6_HEAD_BWD=0 DN_X6_WGRAD1=0";; esac
  env $ev timeout -k 10 200 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/bisect_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -E 'passed|failed' gpurun_out/bisect_$v.log | tail -1)"
  grep -E "^E  .*Error" gpurun_out/bisect_$v.log | head -4
  [ $rc -gt 1 ] && exit $rc
done
exit 0
