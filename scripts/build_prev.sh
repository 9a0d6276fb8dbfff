#!/bin/bash
# Build ncf_amd/libncf_hip_prev.so from the kernel sources at a git revision
# (default HEAD), for A/B timing against the working tree:
#   scripts/build_prev.sh [rev] && python scripts/ab_kernel.py default prev
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/include" "$T/ncf_amd/csrc/build"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" include/); do git -C "$ROOT" show "$REV:$f" > "$T/$f"; done
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" ncf_amd/csrc/ | grep -E '\.(h|hip)$'); do
    git -C "$ROOT" show "$REV:$f" > "$T/$f"
done
cd "$T/ncf_amd/csrc"
for f in ncf_train ncf_ops ncf_layered; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $f.hip -o build/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/ncf_amd/libncf_hip_prev.so" build/*.o
rm -rf "$T"
echo "built ncf_amd/libncf_hip_prev.so from $REV"
