#!/bin/bash
# Regenerates epq_raytracer.patch from a scratch pair of trees (maintainer tool; not run by tests):
#   _work/a = a pristine copy of the reference's src/, _work/b = the same with the patch applied and edited.
#   mkdir -p _work/a _work/b && cp -r /path/to/EPQ_Raytracer/src _work/a/ && cp -r _work/a/src _work/b/ \
#     && (cd _work/b && patch -p1 < ../../epq_raytracer.patch)   # then edit _work/b, then run this
# One line of context per hunk, no timestamps (deterministic output).
set -e
cd "$(dirname "$0")/_work"
diff -Nru -U1 a b | sed -E 's/^((---|\+\+\+) [^\t]+)\t.*$/\1/' > ../epq_raytracer.patch || true
test -s ../epq_raytracer.patch
