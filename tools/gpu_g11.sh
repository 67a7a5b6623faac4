# VO loop kernel trace: per-stream busy / idle per keyframe
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/ptrace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pipe_run.py" 3 40 > "$GRAFT_REPO_ROOT/gpurun_out/ptrace.log" 2>&1) || { tail -20 gpurun_out/ptrace.log; exit 1; }
tail -2 gpurun_out/ptrace.log
timeout -k 10 120 python3 tools/pipe_ktrace.py gpurun_out/ptrace > gpurun_out/ptrace_an.log 2>&1; rc=$?
cat gpurun_out/ptrace_an.log; exit $rc
