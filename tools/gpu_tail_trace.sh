cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r6am_trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/latency_timeline.py" --parts 8 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/r6am_trace.log" 2>&1
