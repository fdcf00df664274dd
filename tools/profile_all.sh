#!/bin/bash
# rocprofv3 evidence for every bench config (tools/profile_round.sh per config), tag given.
# Usage: bash tools/profile_all.sh <tag> [configs...]
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
CONFIGS=${@:-smaq fp8 s2fp8 multi packed smaq_sampled}
for c in $CONFIGS; do
  echo "=== $c"
  bash "$REPO/tools/profile_round.sh" "${TAG}_$c" "$c" 20 3 || exit $?
done
