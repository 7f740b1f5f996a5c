#!/bin/bash
# Round 5: build libgsgpu variants with one tuning constant changed each (sources copied to /tmp,
# nothing in the tree edited) into _var/<name>/libgsgpu.so for a same-box A/B (GSGPU_LIB).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
build() {   # name file sed-expression
  local name=$1 file=$2 expr=$3 d=/tmp/gsvar_$1
  rm -rf "$d"; mkdir -p "$d"
  cp -r "$ROOT/include" "$d/"
  mkdir -p "$d/gelly-streaming_amd"
  cp -r "$ROOT/gelly-streaming_amd/csrc" "$ROOT/gelly-streaming_amd/Makefile" "$d/gelly-streaming_amd/"
  mkdir -p "$d/gelly-streaming_amd/gsgpu/lib" "$d/gelly-streaming_amd/build"
  sed -i "$expr" "$d/gelly-streaming_amd/csrc/$file"
  grep -q "$4" "$d/gelly-streaming_amd/csrc/$file"          # the edit took
  make -C "$d/gelly-streaming_amd" gsgpu/lib/libgsgpu.so > "$d/build.log" 2>&1
  mkdir -p "$ROOT/_var/$name"
  cp "$d/gelly-streaming_amd/gsgpu/lib/libgsgpu.so" "$ROOT/_var/$name/"
  echo "built $name"
}
if [ "${1:-all}" = picks ]; then
build pick64 cc_kernels.hpp 's/kPickEvery = 16;/kPickEvery = 64;/' 'kPickEvery = 64;' &
build admitevery128 cc_kernels.hpp 's/kHotAdmitEvery = 64;/kHotAdmitEvery = 128;/' 'kHotAdmitEvery = 128;' &
wait
exit 0
fi
build admit8 cc_kernels.hpp 's/kHotAdmitLaunches = 4;/kHotAdmitLaunches = 8;/' 'kHotAdmitLaunches = 8;' &
build admit2 cc_kernels.hpp 's/kHotAdmitLaunches = 4;/kHotAdmitLaunches = 2;/' 'kHotAdmitLaunches = 2;' &
build warmat1 cc_api.hip 's/kWarmAt = 2,/kWarmAt = 1,/' 'kWarmAt = 1,' &
build pick32 cc_kernels.hpp 's/kPickEvery = 16;/kPickEvery = 32;/' 'kPickEvery = 32;' &
wait
build thresh2 cc_api.hip 's/kHotThresh = 3;/kHotThresh = 2;/' 'kHotThresh = 2;' &
build cgrid4096 cc_api.hip 's/kCompressGrid = 2048;/kCompressGrid = 4096;/' 'kCompressGrid = 4096;' &
build cgrid1024 cc_api.hip 's/kCompressGrid = 2048;/kCompressGrid = 1024;/' 'kCompressGrid = 1024;' &
wait
