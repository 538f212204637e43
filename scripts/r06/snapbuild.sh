#!/bin/bash
# Build a library from a snapshot of the sources (so editing can continue during the ~5-10 min hipcc run).
# usage: snapbuild.sh <out.so> [extra hipcc flags...]
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$1; shift
SNAP=$(mktemp -d /tmp/kgbuild.XXXXXX)
mkdir -p $SNAP/koordinator_amd $SNAP/include
cp -r $ROOT/koordinator_amd/csrc $SNAP/koordinator_amd/
cp $ROOT/include/*.h $SNAP/include/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result "$@" \
  -shared -o $SNAP/out.so $SNAP/koordinator_amd/csrc/engine.hip -lrccl
mv $SNAP/out.so $OUT
rm -rf $SNAP
echo "built $OUT"
