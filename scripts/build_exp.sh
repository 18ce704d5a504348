#!/bin/bash
# Experiment builds of libdpvo_hot.so: build_exp.sh <name> <extra hipcc flags...>
# -> exp/<name>/libdpvo_hot.so (flavour "<name>": the loader refuses it unless
# DPVO_DIAG=1; load it with DPVO_HOT_LIB).  Never the product.
set -eu
cd "$(dirname "$0")/../wild-video-3d-reconstruction_amd"
name=$1; shift
out=../exp/$name
mkdir -p "$out/obj"
make -s libdpvo_hot.so >/dev/null
SHA=$(cat $(ls csrc/*.hip csrc/*.hpp | sort) ../include/dpvo_hot.h | sha256sum | cut -c1-16)
objs=""
for f in csrc/*.hip; do
  b=$(basename "$f" .hip)
  [ "$b" = buildinfo ] && continue
  ff=""; [ "$b" = altcorr ] && ff="-ffp-contract=off"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result $ff "$@" -c "$f" -o "$out/obj/$b.o" &
  objs="$objs $out/obj/$b.o"
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -DDPVO_SRC_SHA="\"$SHA\"" -DDPVO_EXP_FLAVOUR="\"$name\"" -c csrc/buildinfo.hip -o "$out/obj/buildinfo.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libdpvo_hot.so" $objs "$out/obj/buildinfo.o"
rm -rf "$out/obj"
echo "$out/libdpvo_hot.so"
