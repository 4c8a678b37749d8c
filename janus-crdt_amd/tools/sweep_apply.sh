set -o pipefail
for T in 8 16; do for C in 65536 262144; do
  echo "T=$T C=$C"; JANUS_HOST_THREADS=$T JANUS_WAVE_CHUNK=$C timeout -k 10 120 janus-crdt_amd/build/bench_apply --accounts 1000000 --msgs 1000000 --waves 3 --cpu-msgs 0 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_wave'], d['host_ms_per_wave'], d['engine_ms_per_wave'], d['host_phase_ms'])" || exit 1
done; done
