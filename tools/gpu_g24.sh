# pipeline line under the default bench flags vs --steps 20 --cpu-runs 2 (back to back)
mkdir -p gpurun_out
for a in "" "--steps 20 --cpu-runs 2" ""; do
  timeout -k 10 600 python -u bench.py $a > gpurun_out/b24.json 2> gpurun_out/b24.err || exit 1
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/b24.json') if l.startswith('{')][-1])
p=d['pipeline']; print('args [$a]', d['value'], p['frames_per_s'], p['host_ms_per_frame'], p['wait_ms_per_frame_by_call'])"
done
