#!/usr/bin/env bash
# Build and run the memset-node repro in both HIP graph capture modes (fresh processes).
set -u
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o /tmp/zb_memset_repro memset_repro.hip || exit 2
env -u DEBUG_CLR_GRAPH_PACKET_CAPTURE timeout -k 5 60 /tmp/zb_memset_repro 4
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 5 60 /tmp/zb_memset_repro 4
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 5 60 /tmp/zb_memset_repro 4
exit 0
