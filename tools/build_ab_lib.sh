#!/bin/bash
# Same-box A/B helper: link robustpointclouds_amd/_lib/librpc_hip_ab.so from the current objects with the
# given csrc files taken from git revision REV (run the A/B with RPC_HIP_LIB=<that .so>).
#   tools/build_ab_lib.sh REV spconv.hip [more.hip ...]
set -e
REV=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OBJ=$ROOT/robustpointclouds_amd/_lib/obj
TMP=$(mktemp -d)
mkdir -p $TMP/csrc
cp $ROOT/robustpointclouds_amd/csrc/*.h $TMP/csrc/
OBJS=""
for o in $OBJ/*.hip.o; do
  b=$(basename $o .o)
  skip=0
  for f in "$@"; do [ "$b" = "$f" ] && skip=1; done
  [ $skip -eq 0 ] && OBJS="$OBJS $o"
done
for f in "$@"; do
  git -C $ROOT show $REV:robustpointclouds_amd/csrc/$f > $TMP/csrc/$f
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $ROOT/include -I $TMP/csrc -Wno-unused-result \
    -munsafe-fp-atomics -c $TMP/csrc/$f -o $TMP/$f.o
  OBJS="$OBJS $TMP/$f.o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/robustpointclouds_amd/_lib/librpc_hip_ab.so $OBJS $OBJ/version.o
rm -rf $TMP
echo $ROOT/robustpointclouds_amd/_lib/librpc_hip_ab.so
