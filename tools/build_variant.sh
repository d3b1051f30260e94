#!/bin/bash
# Build the bf16 library with extra compile flags into abvar_<name>/ (git-ignored; travels to the
# GPU box for same-box A/Bs:  STF_LIB=$GRAFT_REPO_ROOT/abvar_<name>/libstfunet_hip.so).
#   bash tools/build_variant.sh <name> "<extra hipcc flags>"
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/stfvar.XXXX)
mkdir -p "$tmp/csrc" "$tmp/stfunet" "$tmp/include" "$root/abvar_$name"
cp "$root"/stf-unet_amd/csrc/*.hip "$root"/stf-unet_amd/csrc/*.h "$root"/stf-unet_amd/csrc/Makefile "$tmp/csrc/"
mkdir -p "$tmp/../include" 2>/dev/null || true
sed -i "s#../../include/stfunet.h#$root/include/stfunet.h#" "$tmp"/csrc/*.hip "$tmp"/csrc/*.h
make -C "$tmp/csrc" -j8 "CXXFLAGS=--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $flags" ../stfunet/libstfunet_hip.so > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
cp "$tmp/stfunet/libstfunet_hip.so" "$root/abvar_$name/"
rm -rf "$tmp"
echo "built abvar_$name/libstfunet_hip.so ($flags)"
