#!/bin/bash
# RCCL over xGMI + RoCE: IOMMU passthrough, no NUMA balancing, large locked memory
set -ex
sudo sed -i 's/GRUB_CMDLINE_LINUX_DEFAULT="/GRUB_CMDLINE_LINUX_DEFAULT="iommu=pt amd_iommu=on /' /etc/default/grub
sudo update-grub
echo 'kernel.numa_balancing=0' | sudo tee /etc/sysctl.d/99-dstack-amd.conf
printf '* soft memlock unlimited\n* hard memlock unlimited\n' | sudo tee /etc/security/limits.d/99-dstack-amd.conf
