"""AWS backend over the EC2 Query API with SigV4 (reference: ``C/backends/aws/compute.py:63-760``,
``resources.py``; the reference uses boto3).

Covers: RunInstances (on-demand/spot, cloud-init shim bootstrap, root volume size, cluster
placement group, capacity reservation, security group with SSH), DescribeInstances polling,
TerminateInstances, placement groups, EBS volumes (create/attach/detach/delete/register) and the
gateway VM.  Config: ``regions``, ``vpc_name``/``subnet_ids``, ``os_images``; creds:
``access_key``/``secret_key`` (or the ``AWS_*`` environment).
"""

from __future__ import annotations

import base64
import os
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.backends.base import choose_disk_size_mib
from dstack_amd.core.backends.clouds.common import VMCompute, check_response, cloud_init, sigv4_headers
from dstack_amd.core.errors import ComputeError, NoCapacityError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gateways import GatewayComputeConfiguration, GatewayProvisioningData
from dstack_amd.core.models.instances import InstanceConfiguration, InstanceOfferWithAvailability
from dstack_amd.core.models.placement import PlacementGroup, PlacementGroupProvisioningData
from dstack_amd.core.models.volumes import Volume, VolumeAttachmentData, VolumeProvisioningData

API_VERSION = "2016-11-15"
UBUNTU_OWNER = "099720109477"
_CAPACITY_CODES = ("InsufficientInstanceCapacity", "InstanceLimitExceeded", "Unsupported",
                   "MaxSpotInstanceCountExceeded", "InsufficientCapacity")


def _strip_ns(root: ET.Element) -> ET.Element:
    for el in root.iter():
        if "}" in el.tag:
            el.tag = el.tag.split("}", 1)[1]
    return root


class AWSCompute(VMCompute):
    TYPE = BackendType.AWS
    SSH_USER = "ubuntu"

    def __init__(self, config: Dict, auth: Dict, client=None):
        super().__init__(config, auth, client)
        self.access_key = self.auth.get("access_key") or os.getenv("AWS_ACCESS_KEY_ID", "")
        self.secret_key = self.auth.get("secret_key") or os.getenv("AWS_SECRET_ACCESS_KEY", "")
        self.session_token = self.auth.get("session_token") or os.getenv("AWS_SESSION_TOKEN")

    # ---- transport ----------------------------------------------------------------------------
    def _call(self, region: str, action: str, params: Optional[Dict[str, str]] = None) -> ET.Element:
        url = f"https://ec2.{region}.amazonaws.com/"
        body = urllib.parse.urlencode({"Action": action, "Version": API_VERSION, **(params or {})}).encode()
        headers = sigv4_headers("POST", url, region, "ec2", self.access_key, self.secret_key, body,
                                self.session_token,
                                extra_headers={"content-type": "application/x-www-form-urlencoded; charset=utf-8"})
        r = self.http.post(url, content=body, headers=headers)
        if r.status_code >= 400:
            root = _strip_ns(ET.fromstring(r.text)) if r.text.startswith("<") else None
            code = root.findtext(".//Code") if root is not None else ""
            msg = root.findtext(".//Message") if root is not None else r.text
            if code in _CAPACITY_CODES:
                raise NoCapacityError(f"{action}: {code}: {msg}")
            check_response(r, f"aws {action} {code}")
        return _strip_ns(ET.fromstring(r.text))

    # ---- helpers ------------------------------------------------------------------------------
    def _image_id(self, region: str, gpu: bool) -> str:
        imgs = self.config.get("os_images") or {}
        key = "amd" if gpu else "cpu"
        if isinstance(imgs.get(key), dict) and imgs[key].get(region):
            return imgs[key][region]
        root = self._call(region, "DescribeImages", {
            "Owner.1": UBUNTU_OWNER, "Filter.1.Name": "name",
            "Filter.1.Value.1": "ubuntu/images/hvm-ssd/ubuntu-jammy-22.04-amd64-server-*",
            "Filter.2.Name": "state", "Filter.2.Value.1": "available"})
        items = [(i.findtext("creationDate") or "", i.findtext("imageId")) for i in root.iter("item")
                 if i.findtext("imageId")]
        if not items:
            raise ComputeError(f"no Ubuntu 22.04 AMI in {region}")
        return max(items)[1]

    def _security_group(self, region: str, project: str) -> str:
        name = f"dstack_{project}"
        root = self._call(region, "DescribeSecurityGroups", {"Filter.1.Name": "group-name", "Filter.1.Value.1": name})
        gid = root.findtext(".//securityGroupInfo/item/groupId")
        if gid:
            return gid
        root = self._call(region, "CreateSecurityGroup", {"GroupName": name, "GroupDescription": "dstack-amd"})
        gid = root.findtext("groupId")
        self._call(region, "AuthorizeSecurityGroupIngress", {
            "GroupId": gid, "IpPermissions.1.IpProtocol": "tcp", "IpPermissions.1.FromPort": "22",
            "IpPermissions.1.ToPort": "22", "IpPermissions.1.IpRanges.1.CidrIp": "0.0.0.0/0"})
        # intra-cluster traffic (RCCL/torchrun between nodes of a fleet)
        self._call(region, "AuthorizeSecurityGroupIngress", {
            "GroupId": gid, "IpPermissions.1.IpProtocol": "-1",
            "IpPermissions.1.Groups.1.GroupId": gid})
        return gid

    # ---- VMCompute hooks ----------------------------------------------------------------------
    def _launch(self, offer: InstanceOfferWithAvailability, cfg: InstanceConfiguration
                ) -> Tuple[str, Optional[str], Optional[dict]]:
        region = offer.region
        res = offer.instance.resources
        params = {
            "ImageId": self._image_id(region, bool(res.gpus)), "InstanceType": offer.instance.name,
            "MinCount": "1", "MaxCount": "1",
            "UserData": base64.b64encode(cloud_init(cfg).encode()).decode(),
            "SecurityGroupId.1": self._security_group(region, cfg.project_name),
            "BlockDeviceMapping.1.DeviceName": "/dev/sda1",
            "BlockDeviceMapping.1.Ebs.VolumeSize": str(max(100, res.disk.size_mib // 1024)),
            "BlockDeviceMapping.1.Ebs.VolumeType": "gp3",
            "TagSpecification.1.ResourceType": "instance",
            "TagSpecification.1.Tag.1.Key": "Name", "TagSpecification.1.Tag.1.Value": cfg.instance_name,
            "TagSpecification.1.Tag.2.Key": "dstack_project", "TagSpecification.1.Tag.2.Value": cfg.project_name,
        }
        if res.spot:
            params["InstanceMarketOptions.MarketType"] = "spot"
            params["InstanceMarketOptions.SpotOptions.SpotInstanceType"] = "one-time"
        if cfg.placement_group_name:
            params["Placement.GroupName"] = cfg.placement_group_name
        if cfg.availability_zone:
            params["Placement.AvailabilityZone"] = cfg.availability_zone
        if cfg.reservation:
            params["CapacityReservationSpecification.CapacityReservationTarget.CapacityReservationId"] = \
                cfg.reservation
        subnets = (self.config.get("subnet_ids") or {}).get(region) if isinstance(self.config.get("subnet_ids"),
                                                                                 dict) else None
        if subnets:
            params["SubnetId"] = subnets
        root = self._call(region, "RunInstances", params)
        iid = root.findtext(".//instancesSet/item/instanceId")
        if not iid:
            raise ComputeError("RunInstances returned no instance id")
        return iid, None, {"region": region}

    def _describe(self, instance_id: str, region: str, backend_data: dict) -> dict:
        root = self._call(region, "DescribeInstances", {"InstanceId.1": instance_id})
        item = root.find(".//instancesSet/item")
        if item is None:
            return {"status": "pending"}
        state = item.findtext("instanceState/name")
        if state in ("terminated", "shutting-down"):
            return {"status": "terminated"}
        return {"status": state, "hostname": item.findtext("ipAddress") or None,
                "internal_ip": item.findtext("privateIpAddress")}

    def _terminate(self, instance_id: str, region: str, backend_data: dict) -> None:
        try:
            self._call(region, "TerminateInstances", {"InstanceId.1": instance_id})
        except ComputeError as e:
            if "InvalidInstanceID.NotFound" not in str(e):
                raise

    # ---- placement groups ---------------------------------------------------------------------
    def create_placement_group(self, placement_group: PlacementGroup) -> PlacementGroupProvisioningData:
        region = placement_group.configuration.region
        self._call(region, "CreatePlacementGroup", {"GroupName": placement_group.name, "Strategy": "cluster"})
        return PlacementGroupProvisioningData(backend=BackendType.AWS)

    def delete_placement_group(self, placement_group: PlacementGroup) -> None:
        self._call(placement_group.configuration.region, "DeletePlacementGroup", {"GroupName": placement_group.name})

    # ---- volumes ------------------------------------------------------------------------------
    def register_volume(self, volume: Volume) -> VolumeProvisioningData:
        root = self._call(volume.configuration.region, "DescribeVolumes",
                          {"VolumeId.1": volume.configuration.volume_id})
        item = root.find(".//volumeSet/item")
        if item is None:
            raise ComputeError(f"volume {volume.configuration.volume_id} not found")
        return VolumeProvisioningData(volume_id=item.findtext("volumeId"), size_gb=int(item.findtext("size") or 0),
                                      availability_zone=item.findtext("availabilityZone"))

    def create_volume(self, volume: Volume) -> VolumeProvisioningData:
        conf = volume.configuration
        zone = getattr(conf, "availability_zone", None) or f"{conf.region}a"
        root = self._call(conf.region, "CreateVolume", {
            "AvailabilityZone": zone, "Size": str(int(conf.size or 100)), "VolumeType": "gp3",
            "TagSpecification.1.ResourceType": "volume", "TagSpecification.1.Tag.1.Key": "Name",
            "TagSpecification.1.Tag.1.Value": volume.name})
        return VolumeProvisioningData(volume_id=root.findtext("volumeId"), size_gb=int(root.findtext("size") or 0),
                                      availability_zone=zone, price=0.08 * float(conf.size or 100) / 730)

    def delete_volume(self, volume: Volume) -> None:
        self._call(volume.configuration.region, "DeleteVolume", {"VolumeId": volume.volume_id})

    def attach_volume(self, volume: Volume, instance_id: str) -> VolumeAttachmentData:
        dev = "/dev/sdf"
        self._call(volume.configuration.region, "AttachVolume",
                   {"VolumeId": volume.volume_id, "InstanceId": instance_id, "Device": dev})
        return VolumeAttachmentData(device_name=dev)

    def detach_volume(self, volume: Volume, instance_id: str, force: bool = False) -> None:
        params = {"VolumeId": volume.volume_id, "InstanceId": instance_id}
        if force:
            params["Force"] = "true"
        self._call(volume.configuration.region, "DetachVolume", params)

    def is_volume_detached(self, volume: Volume, instance_id: str) -> bool:
        root = self._call(volume.configuration.region, "DescribeVolumes", {"VolumeId.1": volume.volume_id})
        return root.find(".//attachmentSet/item") is None

    # ---- gateway ------------------------------------------------------------------------------
    def create_gateway(self, configuration: GatewayComputeConfiguration) -> GatewayProvisioningData:
        from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init

        region = configuration.region
        params = {"ImageId": self._image_id(region, False), "InstanceType": "t3.small", "MinCount": "1",
                  "MaxCount": "1", "UserData": base64.b64encode(gateway_cloud_init(configuration).encode()).decode(),
                  "SecurityGroupId.1": self._gateway_security_group(region, configuration.project_name),
                  "TagSpecification.1.ResourceType": "instance", "TagSpecification.1.Tag.1.Key": "Name",
                  "TagSpecification.1.Tag.1.Value": configuration.instance_name}
        root = self._call(region, "RunInstances", params)
        iid = root.findtext(".//instancesSet/item/instanceId")
        ip = None
        for _ in range(60):
            info = self._describe(iid, region, {})
            if info.get("hostname"):
                ip = info["hostname"]
                break
            import time

            time.sleep(5)
        if ip is None:
            raise ComputeError(f"gateway {iid} got no public IP")
        return GatewayProvisioningData(instance_id=iid, ip_address=ip, region=region)

    def _gateway_security_group(self, region: str, project: str) -> str:
        gid = self._security_group(region, f"{project}_gateway")
        for port in ("80", "443"):
            try:
                self._call(region, "AuthorizeSecurityGroupIngress", {
                    "GroupId": gid, "IpPermissions.1.IpProtocol": "tcp", "IpPermissions.1.FromPort": port,
                    "IpPermissions.1.ToPort": port, "IpPermissions.1.IpRanges.1.CidrIp": "0.0.0.0/0"})
            except ComputeError as e:
                if "Duplicate" not in str(e):
                    raise
        return gid

    def terminate_gateway(self, instance_id: str, configuration: GatewayComputeConfiguration,
                          backend_data: Optional[str] = None) -> None:
        self._terminate(instance_id, configuration.region, {})


_ = (choose_disk_size_mib, List)
