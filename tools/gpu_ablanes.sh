bash tools/ab_quick.sh "--host-path-epochs 0" kafka-matching-engine_amd/kme/libkme.so kafka-matching-engine_amd/kme/libkme_l16w4.so kafka-matching-engine_amd/kme/libkme_l32w3.so
