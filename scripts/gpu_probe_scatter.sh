set -o pipefail
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -Wno-unused-value -Wno-unused-result -o gpurun_out/scatter_probe scripts/probe/scatter_probe.hip
timeout -k 10 120 gpurun_out/scatter_probe > gpurun_out/scatter_probe.jsonl
rm -f gpurun_out/scatter_probe
cat gpurun_out/scatter_probe.jsonl
