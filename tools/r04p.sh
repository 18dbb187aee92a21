# Instruction counts per phase (island, 64-frame launch): base, each phase run twice (tools/exp/
# r04_phase_twice_timing.patch), sky items alone / the rest alone (r04_sky_split_timing.patch).
set -o pipefail
B=epq_raytracer_amd/build
timeout -k 10 900 bash tools/pmc_ab.sh r04p $B/ab_base/libhip_raytrace.so $B/ab_prim2/libhip_raytrace.so \
  $B/ab_bounce2/libhip_raytrace.so $B/ab_shade2/libhip_raytrace.so $B/ab_skyonly/libhip_raytrace.so \
  $B/ab_nonskyonly/libhip_raytrace.so > gpurun_out/r04p_summary.txt 2>&1
