#!/bin/bash
# Build libuavhip.so from a git revision into scripts/<name>/ (A/B baselines; git-ignored, travels
# to the GPU box with gpurun). Usage: bash scripts/build_variant.sh <name> [rev=HEAD] [make args]
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; rev="${2:-HEAD}"; shift 2 || shift $#
tmp=$(mktemp -d)
git -C "$R" archive "$rev" target-allocation-ppo-transformer_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$R/scripts/$name"
make -s -j8 -C "$tmp/target-allocation-ppo-transformer_amd/csrc" BUILD="$tmp/build" OUT="$R/scripts/$name/libuavhip.so" "$@"
rm -rf "$tmp"
