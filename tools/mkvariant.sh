#!/bin/bash
# build one engine variant for tools/ab.py:  tools/mkvariant.sh <name> [hipcc -D/-mllvm flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -Iinclude \
    -mllvm -amdgpu-sched-strategy=iterative-ilp \
    "$@" picotls_amd/csrc/aesgcm_engine.hip -o tools/variants/lib_$name.so
