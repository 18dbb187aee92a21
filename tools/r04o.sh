# Marginal cost of one more dependent round trip: triangle records (L2) and a node step's first member
# pair (LDS); timing-only builds from tools/exp/r04_round_trip_twice_timing.patch.  Island and cave.
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
B=epq_raytracer_amd/build
AB_BATCH=20 timeout -k 10 400 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_tri2/libhip_raytrace.so $B/ab_node2/libhip_raytrace.so > $O/island.jsonl &&
AB_BATCH=20 timeout -k 10 400 bash tools/ab.sh 3 $B/ab_base/libhip_raytrace.so $B/ab_tri2/libhip_raytrace.so $B/ab_node2/libhip_raytrace.so -- --scene cave --node-r 2 > $O/cave.jsonl
