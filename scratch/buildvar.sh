#!/bin/bash
# usage: scratch/buildvar.sh NAME "EXTRA FLAGS"  -> scratch/lib_NAME.so (kernel-variant A/B builds)
set -e
NAME=$1; EXTRA=$2
D=/root/repo/scratch/var_$NAME; mkdir -p $D
SRC=/root/repo/clear-vae_amd/csrc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -w $EXTRA"
ls $SRC/*.hip | xargs -P 16 -I{} sh -c "/opt/rocm/bin/hipcc $FL -c {} -o $D/\$(basename {} .hip).o"
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c $SRC/cv_runtime.cpp -o $D/cv_runtime.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /root/repo/scratch/lib_$NAME.so $D/*.o
echo built scratch/lib_$NAME.so
