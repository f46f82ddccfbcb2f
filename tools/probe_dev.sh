set -o pipefail
echo "== env"; env | grep -i -E 'VISIBLE|ROCR|HIP_|GPU' || true
echo "== dri"; ls -la /dev/dri || true
echo "== kfd dev"; ls -la /dev/kfd || true
echo "== kfd nodes"
for d in /sys/class/kfd/kfd/topology/nodes/*; do echo "$d simd=$(grep -E '^simd_count' $d/properties | awk '{print $2}') gpu_id=$(cat $d/gpu_id 2>/dev/null) drm_render_minor=$(grep drm_render_minor $d/properties | awk '{print $2}')"; done
echo "== cgroup"; cat /proc/self/cgroup; cat /sys/fs/cgroup/devices.list 2>/dev/null || true
echo "== nproc"; nproc
for m in $(ls /dev/dri | grep render); do if [ -r /dev/dri/$m ] && [ -w /dev/dri/$m ]; then echo "rw $m"; else echo "no-access $m"; fi; done
