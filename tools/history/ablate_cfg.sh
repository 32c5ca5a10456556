set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for cfg in "--config 2" "--config 4 --docs 25000000"; do
for a in 0 1 2 8 16 32; do
  LDGPU_LIB=spark-languagedetector_amd/lib/libldgpu_diag.so LDGPU_ABLATE=$a timeout -k 10 200 python3 -u bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-host-path --no-alt-paths > gpurun_out/abl/x.log 2>&1 || { echo "fail $cfg $a"; tail -5 gpurun_out/abl/x.log; exit 1; }
  echo "$cfg ablate=$a $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl/x.log)"
done
done
