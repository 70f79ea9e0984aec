#!/bin/bash
set -ex
curl -fsSL https://get.docker.com | sudo sh
sudo usermod -aG docker ubuntu
# AMD container toolkit: lets `docker run --runtime=amd -e AMD_VISIBLE_DEVICES=...` map GPUs
sudo apt-get install -yqq amd-container-toolkit || true
sudo docker pull rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1
