set -u
for v in base 1 2 8 11; do
  if [ $v = base ]; then L=""; else L="DORKNET_HIP_LIB=$PWD/dorknet_amd/lib/exp$v/libdorknet_hip.so"; fi
  echo "== exp $v"
  env $L timeout -k 10 120 python scripts/pwd_bench.py --deep 1 --only fwd 2>&1 | grep -v amdgpu.ids
  env $L timeout -k 10 120 python scripts/pwd_bench.py --deep 1 --only dgrad 2>&1 | grep -v amdgpu.ids
done
