# Sourced by the GPU scripts: stop the whole call when a log shows a GPU fault
# (the runtime may print one while the process still exits 0).
fault_guard() {
    if grep -q -E "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure" "$@" 2>/dev/null; then
        echo "GPU fault reported in $* -- stopping"
        grep -m3 -E "HSA_STATUS_ERROR|illegal memory access|Memory access fault" "$@"
        exit 86
    fi
}
