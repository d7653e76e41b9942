#!/bin/bash
# Builds the library, surface and tools in-tree until make has nothing left to do; prints errors only.
cd "$(dirname "$0")/.." || exit 1
for i in 1 2 3; do
  make -C p2p-gossipprotocol_amd -j8 > /tmp/gossip_build.log 2>&1 || { grep -E "error" /tmp/gossip_build.log | head -20; exit 1; }
  make -C p2p-gossipprotocol_amd -q && { echo BUILD_OK; exit 0; }
done
echo "build did not settle"; exit 1
