#!/bin/bash
# r05z: frame-run grabs with the pixel pool: grab 4 / tail 64 (ab_pbase = product), grab 8, grab 8 tail 32,
# tail 32, tail 16 -- whole frame + rank 6 of 8 at bench.py's shape, island and cave x2, interleaved.
set -o pipefail
OUT=gpurun_out/r05z; mkdir -p $OUT
B=epq_raytracer_amd/build
for r in 1 2; do
  for S in island cave; do
    for L in pbase g8 g8t32 t32 t16; do
      HRT_LIB=$B/ab_$L/libhip_raytrace.so timeout -k 10 150 python3 tools/rank_shape.py --rounds 1 --parts 6 --scene $S > $OUT/rs.jsonl 2>&1 || { echo "rank shape $L $S failed"; tail -5 $OUT/rs.jsonl; exit 1; }
      echo "$r $L $(tail -1 $OUT/rs.jsonl)" | tee -a $OUT/rank_ab.txt
    done
  done
done
