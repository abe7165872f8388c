#!/bin/bash
# build an experiment variant of libnerf_amd.so into exp/<name>.so with extra -D flags for mlp_bf16.hip the NGP/MoE/meta sources, adam.hip and mlp.hip
# usage: tools/build_exp.sh NAME "-DFOO -DBAR" [OVERRIDE_DIR]
#   OVERRIDE_DIR: files in it replace the same-named csrc files (a candidate header compared against the committed one)
set -e
cd "$(dirname "$0")/../nerf-sys_amd"
rm -rf /tmp/exp_$1; mkdir -p ../exp /tmp/exp_$1
SRC=csrc
if [ -n "$3" ]; then  # csrc includes ../../include/nerf_amd.h: keep that relative path valid in the copy
  R=/tmp/exp_src_$1; rm -rf $R; mkdir -p $R/pkg; cp -r csrc $R/pkg/csrc; ln -s "$PWD/../include" $R/include
  SRC=$R/pkg/csrc; cp "$3"/* $SRC/
fi
for f in $SRC/*.hip; do
  b=$(basename $f .hip); X=""
  [ $b = mlp_bf16 ] && X="-mllvm -disable-promote-alloca-to-lds $2"
  { [ $b = ngp ] || [ $b = moe ] || [ $b = meta ]; } && X="-ffp-contract=off $2"
  { [ $b = adam ] || [ $b = mlp ]; } && X="$2"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $X -c $f -o /tmp/exp_$1/$b.o &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds -DNERF_F16=1 $2 -c $SRC/mlp_bf16.hip -o /tmp/exp_$1/mlp_f16.o &
for j in $(jobs -p); do wait $j; done
echo "extern \"C\" const char* nerf_version(void) { return \"nerf_amd 0.2 gfx950 src=exp-$1\"; }" > /tmp/exp_$1/version.cpp
g++ -O2 -fPIC -c /tmp/exp_$1/version.cpp -o /tmp/exp_$1/version.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 /tmp/exp_$1/*.o -o ../exp/$1.so
echo built exp/$1.so
