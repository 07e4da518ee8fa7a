set -e
mkdir -p gpurun_out
for e in "X=0" "DEBUG_CLR_SKIP_RELEASE_SCOPE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "ROC_SYSTEM_SCOPE_SIGNAL=0"; do
  echo "== $e" >> gpurun_out/envprobe.txt
  env $e timeout -k 10 90 python -u scripts/launch_gap_probe.py >> gpurun_out/envprobe.txt 2>&1
done
