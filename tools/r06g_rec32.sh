#!/bin/bash
# Band records (tools/exp/r05w_band_records_rejected.patch) re-measured on this round's kernel: time (A/B)
# and the counter traffic (FETCH_SIZE / WRITE_SIZE passes) of both builds, island and cave.
set -o pipefail
bash tools/r06_ab.sh r06g 3 rec32 || exit 1
B=epq_raytracer_amd/lib/libhip_raytrace.so; R=epq_raytracer_amd/build/ab_rec32/libhip_raytrace.so
PMC="FETCH_SIZE" bash tools/pmc_ab.sh r06g_fetch_island $B $R || exit 1
PMC="WRITE_SIZE" bash tools/pmc_ab.sh r06g_write_island $B $R || exit 1
PMC="FETCH_SIZE" FRAMES_ARGS="--scene cave" bash tools/pmc_ab.sh r06g_fetch_cave $B $R || exit 1
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY" bash tools/pmc_ab.sh r06g_inst_island $B $R || exit 1
