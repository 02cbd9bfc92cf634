#!/bin/bash
# Is a CPU Vulkan implementation (Mesa lavapipe) available to run the reference renderer as the CPU
# baseline? Lists Vulkan ICD manifests, loader / lavapipe libraries and tools. Output: $1 (default
# gpurun_out/vulkan_probe.txt).
out=${1:-gpurun_out/vulkan_probe.txt}
mkdir -p "$(dirname "$out")"
{
  echo "# host: $(uname -srm); $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2 | sed 's/^ //'); nproc=$(nproc)"
  echo "# date: $(date -u +%FT%TZ)"
  for d in /usr/share/vulkan/icd.d /etc/vulkan/icd.d /usr/local/share/vulkan/icd.d "$HOME/.local/share/vulkan/icd.d"; do
    if [ -d "$d" ]; then echo "ICD dir $d:"; ls -la "$d"; else echo "ICD dir $d: absent"; fi
  done
  echo "VK_ICD_FILENAMES=${VK_ICD_FILENAMES:-<unset>} VK_DRIVER_FILES=${VK_DRIVER_FILES:-<unset>}"
  echo "ldconfig entries matching vulkan|lvp|mesa:"
  ldconfig -p | grep -i -E "vulkan|lvp|mesa" || echo "  (none)"
  echo "libvulkan_lvp.so / libvulkan.so on disk:"
  timeout 60 find / -xdev \( -name 'libvulkan_lvp.so*' -o -name 'libvulkan.so*' -o -name 'lvp_icd*.json' \) 2>/dev/null | head -20 || true
  [ -z "$(timeout 60 find / -xdev \( -name 'libvulkan_lvp.so*' -o -name 'libvulkan.so*' \) 2>/dev/null | head -1)" ] && echo "  (none)"
  echo "tools: vulkaninfo=$(command -v vulkaninfo || echo absent) glslangValidator=$(command -v glslangValidator || echo absent) glslc=$(command -v glslc || echo absent)"
} > "$out" 2>&1
cat "$out"
