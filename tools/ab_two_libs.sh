# A/B of two library builds in separate processes: usage bash tools/ab_two_libs.sh <script> <libA> <libB>
# (each lib is copied over the in-tree libsfmhip.so before its run; the product lib ab/lib_prod.so
# is restored at the end).  Three alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=3d_reconstruction_amd/libsfmhip.so
S=$1; A=$2; B=$3
for rep in 1 2 3; do
  for lib in $A $B; do
    cp $lib $L
    echo -n "$(basename $lib) "; timeout -k 10 120 python $S 2>/dev/null | tail -1 || { cp ab/lib_prod.so $L; exit 1; }
  done
done
cp ab/lib_prod.so $L
