#!/bin/bash
# Builds an A/B variant of libnwc.so with extra compile flags (e.g. -DNWC_VERIFY_WAVES_PER_SIMD=3)
# into narwhal_amd/variants/<name>.so (git-ignored, travels to the GPU box with the tree).
#   tools/build_variant.sh <name> [hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p $R/narwhal_amd/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -shared -I$R/include -I$R/narwhal_amd/csrc "$@" \
  -o $R/narwhal_amd/variants/$NAME.so $R/narwhal_amd/csrc/nwc_api.hip
echo built narwhal_amd/variants/$NAME.so
