#!/bin/bash
# Copy the scratch working copy's sources (.wt, edited while a GPU call holds a
# snapshot of the tree) back into the tree: csrc, include, the Python package,
# tests, scripts, bench.py, the graft entry.  Then rebuild the library.
set -eu
cd "$(dirname "$0")/.."
for d in fast-slam_amd/csrc include fast-slam_amd/fast_slam_2 tests scripts oracle; do
  (cd .wt && find "$d" -type f \( -name '*.hip' -o -name '*.hpp' -o -name '*.h' -o -name '*.py' -o -name '*.sh' -o -name '*.c' -o -name 'Makefile' \) -print) |
  while read -r f; do
    if ! cmp -s ".wt/$f" "$f"; then mkdir -p "$(dirname "$f")"; cp ".wt/$f" "$f"; echo "synced $f"; fi
  done
done
for f in bench.py __graft_entry__.py fast-slam_amd/build.py fast-slam_amd/fs2_synthetic.py; do
  if ! cmp -s ".wt/$f" "$f"; then cp ".wt/$f" "$f"; echo "synced $f"; fi
done
python fast-slam_amd/build.py > /dev/null
