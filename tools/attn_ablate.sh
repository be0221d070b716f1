#!/bin/bash
# Build ablation variants of the library (attention.hip with -DATTN_ABL=k) under exp/ for
# tools/opbench.py --lib; the product library is untouched.
set -e
cd "$(dirname "$0")/.."
PKG=video-latent-diffusion-panoptic-segmentation_amd
mkdir -p exp
objs=$(ls $PKG/build/*.o | grep -v '/attention.o$')
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -DATTN_ABL=$k -c $PKG/csrc/attention.hip -o exp/attention_abl$k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs exp/attention_abl$k.o -o exp/libabl$k.so
  echo "exp/libabl$k.so"
done
