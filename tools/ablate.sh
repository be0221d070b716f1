#!/bin/bash
# Build an ablation variant of the library: one source recompiled with extra -D flags, linked
# with the other objects into ablx/lib<tag>.so, for tools/opbench.py --lib.  The product
# library is untouched.   usage: tools/ablate.sh <tag> <source.hip> -DNAME=VAL ...
set -e
cd "$(dirname "$0")/.."
PKG=video-latent-diffusion-panoptic-segmentation_amd
tag=$1; src=$2; shift 2
mkdir -p ablx
base=$(basename "$src" .hip)
objs=$(ls $PKG/build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude "$@" -c "$src" -o ablx/${base}_$tag.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs ablx/${base}_$tag.o -o ablx/lib$tag.so
echo "ablx/lib$tag.so"
