#!/bin/bash
# Build a variant library that differs from the in-tree one only in cv_direct.hip:
#   tools/build_variant.sh OUT.so SOURCE.hip [extra hipcc flags...]     (run from the repo root, after `make`)
OUT=$1; SRC=$2; shift 2
D=clear-vae_amd/csrc
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Wall -Wno-unused-variable -Wno-unused-but-set-variable -Wno-unused-function"
cp "$SRC" $D/.variant_direct.hip
/opt/rocm/bin/hipcc $HF "$@" -I$D -Iinclude -c $D/.variant_direct.hip -o /tmp/variant_direct.o || exit 1
rm -f $D/.variant_direct.hip
OBJS=$(ls $D/*.o | grep -v "stamps\|cv_direct.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" /tmp/variant_direct.o $OBJS && echo "built $OUT"
