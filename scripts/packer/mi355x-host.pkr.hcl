# Host image for MI355X nodes (reference: scripts/packer/* — docker + nvidia toolkit + CUDA).
# Installs the ROCm kernel driver + amd-smi, Docker, the AMD container toolkit, kernel tweaks for
# RCCL over xGMI/RoCE, pre-pulls the base image, and installs dstack-shim as a systemd service.
variable "base_ami"   { type = string }
variable "region"     { type = string }
variable "rocm_version" { default = "6.4" }

source "amazon-ebs" "mi355x" {
  ami_name      = "dstack-amd-mi355x-rocm${var.rocm_version}-{{timestamp}}"
  instance_type = "c6i.2xlarge"
  region        = var.region
  source_ami    = var.base_ami
  ssh_username  = "ubuntu"
}

build {
  sources = ["source.amazon-ebs.mi355x"]
  provisioner "shell" {
    scripts = ["provisioners/rocm.sh", "provisioners/docker.sh", "provisioners/kernel-tuning.sh",
               "provisioners/dstack-shim.sh"]
    environment_vars = ["ROCM_VERSION=${var.rocm_version}"]
  }
}
