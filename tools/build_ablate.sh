#!/bin/bash
# Variant library with extra flags on some translation units (diagnostic builds, e.g. -DCV_ABLATE=4 on the bf16
# GEMM-core units):  tools/build_ablate.sh OUT.so "unit1.hip unit2.hip" [hipcc flags...]   (repo root, after make)
OUT=$1; UNITS=$2; shift 2
D=clear-vae_amd/csrc
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Wall -Wno-unused-variable -Wno-unused-but-set-variable -Wno-unused-function"
mkdir -p /tmp/abl && rm -f /tmp/abl/*.o
EX=""
for u in $UNITS; do
  b=$(basename $u .hip)
  /opt/rocm/bin/hipcc $HF "$@" -I$D -Iinclude -c $D/$u -o /tmp/abl/$b.o || exit 1
  EX="$EX\|$b.o"
done
OBJS=$(ls $D/*.o | grep -v "stamps$EX")
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" /tmp/abl/*.o $OBJS && echo "built $OUT"
