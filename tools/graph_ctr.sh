#!/bin/bash
# Arrival-counter path (deferral off) eager vs captured in one graph, with the graph-safe device
# stream counter (DS_CTR=1), and deferral on in a graph.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export DS_SIZES=1048576,4194304,16777216 DS_CALLS=60
echo "== eager, deferral off, ctr"; SMQ_DEFER_MAX_N=0 DS_CTR=1 timeout -k 10 120 python tools/defer_sweep.py || exit 1
echo "== graph, deferral off, ctr"; SMQ_DEFER_MAX_N=0 DS_CTR=1 DS_GRAPH=1 timeout -k 10 120 python tools/defer_sweep.py || exit 1
echo "== graph, deferral on, ctr"; DS_CTR=1 DS_GRAPH=1 timeout -k 10 120 python tools/defer_sweep.py || exit 1
