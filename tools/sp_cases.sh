mkdir -p gpurun_out/sp
GAR_BG_TRACE=1 SP_CASE=11025,176400,2,F64,4096 timeout -k 10 200 python -u tools/seam_probe.py > gpurun_out/sp/trace.log 2>&1 || exit 1
for c in 11025,176400,1,F64,4096 11025,176400,3,F64,4096 11025,176400,4,F64,4096 11025,176400,7,F64,4096 8000,128000,2,F64,4096 22050,176400,2,F64,4096 11025,88200,2,F64,4096 11025,44100,2,F64,4096 48000,96000,2,F64,4096 11025,176400,2,F32_EXACT,4096; do
  echo "== $c" >> gpurun_out/sp/cases.log
  SP_CASE=$c timeout -k 10 200 python -u tools/seam_probe.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/sp/cases.log || exit 1
done
