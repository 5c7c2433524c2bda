cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
C="c_raytracer:960x540x16/8,world:960x540x16/8"
for cfg in "RT_AMD_SERIAL_Z10=12" "RT_AMD_SERIAL_Z10=18" "RT_AMD_SERIAL_Z10=21" "RT_AMD_SERIAL_Z10=15" "RT_AMD_SERIAL_EST=256" "RT_AMD_SERIAL_CHUNK=98304"; do
  echo "== $cfg" >> gpurun_out/sweep3.log
  env $cfg REPS=2 CASES="$C" timeout -k 10 200 python -u tools/serial_probe.py >> gpurun_out/sweep3.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/sweep3.log
