# A/B of the single pass's line stores (nontemporal / plain): timing and WRITE_SIZE
set -e
QB_N=1048576 tools/ab.sh 2,4 build/variants/cur.so@5 build/variants/spp.so@5 build/variants/cur.so@5 build/variants/spp.so@5 > gpurun_out/r5AL_sp_plain.log 2>&1
export TMPDIR=/tmp
for v in cur spp; do
  cp build/variants/$v.so capnproto-java_amd/lib/libcapnp_packed_hip.so
  for c in 2 4; do
    timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r5AL_w_${v}_$c -o w --output-format csv -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > gpurun_out/r5AL_w_${v}_$c.log 2>&1
  done
done
echo done >> gpurun_out/r5AL_sp_plain.log
