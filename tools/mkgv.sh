#!/bin/bash
# build one engine variant for the round-5 GPU recipes: tools/mkgv.sh <name> [hipcc -D flags...]
#   -> tools/gv/<name>/libptls_mi355x.so (a directory per variant, so LD_LIBRARY_PATH can select it for the C tests)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/gv/$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value -Iinclude \
    -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" picotls_amd/csrc/aesgcm_engine.hip -o tools/gv/$name/libptls_mi355x.so
