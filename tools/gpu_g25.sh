# scale LM worker on the C call only: pipeline GPU tests, loop timing x3, default bench x2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/t25.log 2>&1 || { tail -20 gpurun_out/t25.log; exit 1; }
tail -1 gpurun_out/t25.log
for r in 1 2 3; do timeout -k 10 200 python3 tools/pipe_run.py 3 40 2>/dev/null | grep -E "^config" || exit 1; done
for r in 1 2; do
  timeout -k 10 600 python -u bench.py > gpurun_out/b25.json 2> gpurun_out/b25.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b25.json') if l.startswith('{')][-1])
p=d['pipeline']; q=d['pipeline_config5']; print(d['value'], p['frames_per_s'], p['host_ms_per_frame'], p['wait_ms_per_frame_by_call'], q['frames_per_s'], p['parity']['events_bit_exact'], q['parity']['ok'])"
done
