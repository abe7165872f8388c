#!/bin/bash
# build an experiment variant of libnerf_amd.so into exp/<name>.so with extra -D flags for mlp_bf16.hip the NGP/MoE/meta sources, adam.hip and mlp.hip
# usage: tools/build_exp.sh NAME "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../nerf-sys_amd"
mkdir -p ../exp /tmp/exp_$1
for f in csrc/*.hip; do
  b=$(basename $f .hip); X=""
  [ $b = mlp_bf16 ] && X="-mllvm -disable-promote-alloca-to-lds $2"
  { [ $b = ngp ] || [ $b = moe ] || [ $b = meta ]; } && X="-ffp-contract=off $2"
  { [ $b = adam ] || [ $b = mlp ]; } && X="$2"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $X -c $f -o /tmp/exp_$1/$b.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 /tmp/exp_$1/*.o -o ../exp/$1.so
echo built exp/$1.so
