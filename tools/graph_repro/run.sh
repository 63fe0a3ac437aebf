#!/usr/bin/env bash
# Build and run the HIP-graph kernel-argument repro with packet capture on (the CLR default) and off.
# Usage (GPU box): bash tools/graph_repro/run.sh
set -u
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o /tmp/zb_graph_repro repro.hip || exit 2
for kind in small big; do
  for n in 0 1 64 4096; do
    env -u DEBUG_CLR_GRAPH_PACKET_CAPTURE timeout -k 5 60 /tmp/zb_graph_repro $n $kind
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 5 60 /tmp/zb_graph_repro $n $kind
  done
done
exit 0
