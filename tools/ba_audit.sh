# BA kernel audit: the product build of ba_trf_kernel against two tool-only
# builds of the same source (abl/lib_ba_audit.so: -DSFMHIP_BA_AUDIT, a full wait + barrier at every
# phase boundary; abl/lib_ba_printf.so: -DSFMHIP_BA_PRINTF, an inert printf in every pass), each run
# twice, alternating, on the bench's 256-pair x 4096-observation BA batch: every run must print the
# same output digest (cam, X, nfev, njev, cost).  abl/lib_prod.so is restored at the end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=3d_reconstruction_amd/libsfmhip.so
for rep in 1 2; do
  for v in prod ba_audit ba_printf; do
    cp abl/lib_$v.so $L
    echo -n "$v: "; timeout -k 10 120 python tools/ba_probe.py 256 | grep "pairs:" || { cp abl/lib_prod.so $L; exit 1; }
  done
done
cp abl/lib_prod.so $L
