#!/bin/bash
set -ex
sudo apt-get update -qq
wget -q "https://repo.radeon.com/amdgpu-install/${ROCM_VERSION}/ubuntu/jammy/amdgpu-install_${ROCM_VERSION}.60400-1_all.deb" -O /tmp/amdgpu-install.deb
sudo apt-get install -yqq /tmp/amdgpu-install.deb
sudo amdgpu-install -y --usecase=dkms,rocm --no-32
sudo usermod -aG render,video ubuntu
