#!/bin/bash
# Record the git state of this tree in .tree_stamp before a GPU call (the box's snapshot has no
# .git): head commit, and "+dirty" with a hash of the uncommitted diff when there is one.
cd "$(dirname "$0")/.."
h=$(git rev-parse HEAD)
if git diff --quiet HEAD -- . ':!.tree_stamp'; then
  echo "$h" > .tree_stamp
else
  echo "$h+dirty:$(git diff HEAD -- . ':!.tree_stamp' | sha256sum | cut -c1-12)" > .tree_stamp
fi
cat .tree_stamp
