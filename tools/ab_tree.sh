#!/bin/bash
# Whole-tree A/B baseline: git revision $1 (default HEAD) exported to ./abase and its library built there;
# a GPU script then runs `python abase/bench.py` beside `python bench.py` in the same call.
set -e
REV=${1:-HEAD}
cd "$(dirname "$0")/.."
rm -rf abase && mkdir abase
git archive "$REV" bench.py __graft_entry__.py include oracle tools vit-of-pytorch_amd | tar -x -C abase
make -C abase/vit-of-pytorch_amd -j8 > /tmp/abase_build.log 2>&1
echo "abase: $(git rev-parse --short $REV)"
