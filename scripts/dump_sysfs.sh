# Capture the GPU box's KFD topology / DRM layout as test fixtures (read-only).
out=gpurun_out/sysfs
mkdir -p $out
T=/sys/class/kfd/kfd/topology
{
  echo "generation_id $(cat $T/generation_id 2>/dev/null)"
  echo "system_properties:"; cat $T/system_properties 2>/dev/null
} > $out/topology_top.txt
for n in $T/nodes/*; do
  id=$(basename $n); d=$out/nodes/$id; mkdir -p $d
  cp $n/properties $d/properties 2>/dev/null
  cat $n/name > $d/name 2>/dev/null
  cat $n/gpu_id > $d/gpu_id 2>/dev/null
  for l in $n/io_links/* $n/p2p_links/*; do
    [ -e "$l/properties" ] || continue
    k=$(basename $(dirname $l))/$(basename $l); mkdir -p $d/$k; cp $l/properties $d/$k/properties
  done
  for m in $n/mem_banks/*; do
    [ -e "$m/properties" ] || continue
    mkdir -p $d/mem_banks/$(basename $m); cp $m/properties $d/mem_banks/$(basename $m)/properties
  done
done
ls -la /dev/dri /dev/kfd > $out/dev_ls.txt 2>&1
for r in /sys/class/drm/renderD* /sys/class/drm/card*; do echo "$r -> $(readlink -f $r/device)"; done > $out/drm_links.txt 2>&1
for r in /sys/class/drm/renderD*; do p=$(readlink -f $r/device); echo "$(basename $r) numa=$(cat $p/numa_node 2>/dev/null) vendor=$(cat $p/vendor 2>/dev/null) device=$(cat $p/device 2>/dev/null)"; done > $out/drm_pci.txt 2>&1
(command -v amd-smi && timeout 60 amd-smi list) > $out/amd_smi_list.txt 2>&1
(timeout 60 amd-smi topology) > $out/amd_smi_topo.txt 2>&1
(timeout 60 rocminfo | head -150) > $out/rocminfo.txt 2>&1
(timeout 120 rocprofv3 -L) > $out/rocprof_counters.txt 2>&1
id > $out/id.txt; env | grep -iE "HIP|ROCR|CUDA|HSA|GPU" > $out/env.txt
echo ok
