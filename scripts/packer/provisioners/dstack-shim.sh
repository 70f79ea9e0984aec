#!/bin/bash
set -ex
sudo curl -fsSL -o /usr/local/bin/dstack-shim "${DSTACK_SHIM_DOWNLOAD_URL:-https://dstack-amd-releases.s3.amazonaws.com/latest/dstack-shim-linux-amd64}"
sudo chmod +x /usr/local/bin/dstack-shim
sudo tee /etc/systemd/system/dstack-shim.service >/dev/null <<'UNIT'
[Unit]
Description=dstack-amd shim
After=network.target docker.service
[Service]
ExecStart=/usr/local/bin/dstack-shim --service --driver auto
Restart=always
[Install]
WantedBy=multi-user.target
UNIT
sudo systemctl enable dstack-shim
