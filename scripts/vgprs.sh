#!/bin/bash
# VGPRs / scratch bytes per lane of every fused train-step kernel instance (host-side check).
cd "$(dirname "$0")/../ncf_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage \
    -c ncf_train.hip -o /tmp/ncf_vgprs.o 2>&1 |
    grep -E "Function Name|VGPRs:|ScratchSize" | paste - - - | grep "Lb0" |
    sed -E 's/.*ncf_step_kernelILi([0-9]+)ELi([0-9]+)ELi([0-9]+)ELb0.*VGPRs: ([0-9]+).*lane\]: ([0-9]+).*/F=\1 L=\2 mode=\3 vgpr=\4 scratch=\5/'
