#!/bin/bash
# Rebuild the in-tree hiprtc code-object cache for the prebuilt pattern sets
# (build() and tools/prebuild_tests.py) and delete every object neither of them
# wrote or read (a cache hit refreshes the file's time): the objects of older
# sources would otherwise travel to the GPU box with every call.
set -eu
cd "$(dirname "$0")/.."
cache=telomere-analyzer_amd/nanotel_amd/jitcache
stamp=$(mktemp)
sleep 1
python -c "import __graft_entry__ as g; g.build()"
python tools/prebuild_tests.py
n0=$(ls "$cache" | wc -l)
find "$cache" -name 'nt_*.co' ! -newer "$stamp" -delete
rm -f "$stamp"
echo "jit cache: $n0 -> $(ls "$cache" | wc -l) objects"
