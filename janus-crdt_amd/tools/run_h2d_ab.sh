S=janus-crdt_amd/tools/gpu_steps.sh
B="janus-crdt_amd/build/bench_apply --accounts 1000000 --ops 1000000 --waves 3 --cpu-msgs 0 --device 0"
bash $S h2d.log 100 janus-crdt_amd/build/tune_h2d && HSA_ENABLE_SDMA=0 bash $S h2d_blit.log 100 janus-crdt_amd/build/tune_h2d && \
JANUS_H2D_SPLIT=0 bash $S ap_s0a.log 120 $B && JANUS_H2D_SPLIT=1 bash $S ap_s1a.log 120 $B && JANUS_H2D_SPLIT=0 bash $S ap_s0b.log 120 $B && JANUS_H2D_SPLIT=1 bash $S ap_s1b.log 120 $B && \
bash $S tune_grouped.log 150 janus-crdt_amd/build/tune_grouped
