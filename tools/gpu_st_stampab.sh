#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for b in build/st_stamps build/st_stamps_ab1 build/st_stamps_ab2 build/st_stamps_ab3 build/st_stamps_ab4; do
  [ -x $b ] || continue
  echo "== $b"; timeout -k 10 60 $b 2>&1 | grep -E "waves|K=3|lifetime|encode|decode" || exit 1
done
