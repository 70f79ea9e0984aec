"""AWS backend over the EC2 Query API with SigV4 (reference: ``C/backends/aws/compute.py:63-760``,
``resources.py``; the reference uses boto3).

Covers: RunInstances (on-demand/spot, cloud-init shim bootstrap, root volume size, cluster
placement group, capacity reservations and capacity blocks, tags), VPC selection (default VPC,
``vpc_name`` tag lookup or ``vpc_ids``, configured ``subnet_ids``, public-IP subnets), one attempt
per availability zone on no-capacity, EFA network interfaces sized from DescribeInstanceTypes
(``efa`` / ``efa-only`` cards for RCCL's inter-node RDMA), paginated Describe* calls,
DescribeInstances polling (private address when ``public_ips: false``), TerminateInstances,
placement groups, EBS volumes (create/attach/detach/delete/register) and the gateway VM.
Config: ``regions``, ``vpc_name``/``vpc_ids``/``subnet_ids``, ``public_ips``, ``os_images``,
``tags``; creds: ``access_key``/``secret_key`` (or the ``AWS_*`` environment).
"""

from __future__ import annotations

import base64
import concurrent.futures as cf
import datetime as _dt
import json
import logging
import os
import urllib.parse
import xml.etree.ElementTree as ET
from dataclasses import replace
from typing import Dict, List, Optional, Set, Tuple

from dstack_amd.core.backends.catalog import CatalogRow, offline_rows
from dstack_amd.core.backends.clouds.common import VMCompute, check_response, cloud_init, sigv4_headers
from dstack_amd.core.backends.clouds.tags import merged_tags
from dstack_amd.core.errors import BackendAuthError, ComputeError, ComputeResourceNotFoundError, NoCapacityError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gateways import GatewayComputeConfiguration, GatewayProvisioningData
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
)
from dstack_amd.core.models.placement import PlacementGroup, PlacementGroupProvisioningData
from dstack_amd.core.models.volumes import Volume, VolumeAttachmentData, VolumeProvisioningData

logger = logging.getLogger(__name__)

API_VERSION = "2016-11-15"
UBUNTU_OWNER = "099720109477"
_CAPACITY_CODES = ("InsufficientInstanceCapacity", "InstanceLimitExceeded", "Unsupported",
                   "MaxSpotInstanceCountExceeded", "InsufficientCapacity")


def _strip_ns(root: ET.Element) -> ET.Element:
    for el in root.iter():
        if "}" in el.tag:
            el.tag = el.tag.split("}", 1)[1]
    return root


def quota_class(instance_name: str, spot: bool) -> str:
    """EC2 vCPU quota class of an instance type (the ``Class`` dimension of the service quota's
    usage metric: ``P/OnDemand``, ``G/Spot``, ``Standard/OnDemand``, ...)."""
    fam = instance_name.split(".")[0].lower()
    for prefix, cls in (("trn", "Trn"), ("inf", "Inf"), ("dl", "DL"), ("vt", "G"), ("p", "P"), ("g", "G"),
                        ("x", "X"), ("f", "F")):
        if fam.startswith(prefix):
            return f"{cls}/{'Spot' if spot else 'OnDemand'}"
    return f"Standard/{'Spot' if spot else 'OnDemand'}"


class AWSCompute(VMCompute):
    TYPE = BackendType.AWS
    SSH_USER = "ubuntu"
    CONFIGURABLE_DISK = (1.0, 16384.0)  # EBS gp2/gp3 root volume, GiB

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

    def _paginate(self, region: str, action: str, params: Optional[Dict[str, str]], item_path: str) -> List[ET.Element]:
        """All items of a paginated Describe* call (follows ``nextToken``)."""
        items: List[ET.Element] = []
        token = None
        for _ in range(100):
            p = dict(params or {})
            if token:
                p["NextToken"] = token
            root = self._call(region, action, p)
            items.extend(root.findall(item_path))
            token = root.findtext("nextToken")
            if not token:
                break
        return items

    def check_credentials(self) -> None:
        """STS GetCallerIdentity: valid for any credentials that can sign, whatever their policies."""
        url = "https://sts.amazonaws.com/"
        body = urllib.parse.urlencode({"Action": "GetCallerIdentity", "Version": "2011-06-15"}).encode()
        headers = sigv4_headers("POST", url, "us-east-1", "sts", self.access_key, self.secret_key, body,
                                self.session_token,
                                extra_headers={"content-type": "application/x-www-form-urlencoded; charset=utf-8"})
        r = self.http.post(url, content=body, headers=headers)
        if r.status_code in (400, 401, 403):
            raise BackendAuthError(f"aws sts: {r.status_code} {r.text[:300]}")
        check_response(r, "aws sts")

    # ---- live catalog -------------------------------------------------------------------------
    def _fetch_catalog(self) -> List[CatalogRow]:
        """Catalog rows checked against the account, per region (reference ``get_offers``,
        ``aws/compute.py:105-141``): instance types not offered in the region are
        ``not_available``, types whose vCPU quota class is below the type's vCPUs are ``no_quota``,
        spot rows take the current lowest spot price over the region's zones."""
        base = offline_rows(self.TYPE)
        wanted = self.config.get("regions")
        regions = sorted({r.location for r in base if not wanted or r.location in wanted})
        names = sorted({r.instance_name for r in base})
        with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(regions)))) as ex:
            info = dict(zip(regions, ex.map(lambda reg: self._region_catalog(reg, names), regions)))
        out = []
        for r in base:
            if r.location not in info:
                continue
            offered, spot_prices, quotas = info[r.location]
            if r.instance_name not in offered:
                out.append(replace(r, availability=InstanceAvailability.NOT_AVAILABLE))
                continue
            price = spot_prices.get(r.instance_name, r.price) if r.spot else r.price
            quota = quotas.get(quota_class(r.instance_name, r.spot)) if quotas is not None else None
            avail = InstanceAvailability.NO_QUOTA if quota is not None and quota < r.cpu else \
                InstanceAvailability.UNKNOWN
            out.append(replace(r, price=round(price, 6), availability=avail))
        return out

    def _region_catalog(self, region: str, names: List[str]
                        ) -> Tuple[Set[str], Dict[str, float], Optional[Dict[str, float]]]:
        params = {"LocationType": "region", "Filter.1.Name": "instance-type"}
        for i, n in enumerate(names, 1):
            params[f"Filter.1.Value.{i}"] = n
        offered = {it.findtext("instanceType") for it in self._paginate(
            region, "DescribeInstanceTypeOfferings", params, "./instanceTypeOfferingSet/item")}
        sp = {"ProductDescription.1": "Linux/UNIX",
              "StartTime": _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")}
        for i, n in enumerate(sorted(offered), 1):
            sp[f"InstanceType.{i}"] = n
        spot: Dict[str, float] = {}
        if offered:
            for it in self._paginate(region, "DescribeSpotPriceHistory", sp, "./spotPriceHistorySet/item"):
                t, price = it.findtext("instanceType"), float(it.findtext("spotPrice") or "inf")
                spot[t] = min(price, spot.get(t, price))
        return offered, spot, self._quotas(region)

    def _quotas(self, region: str) -> Optional[Dict[str, float]]:
        """vCPU quotas by class from Service Quotas (``None`` when the API is not permitted: the
        rows then keep ``unknown`` availability, as without quota information)."""
        url = f"https://servicequotas.{region}.amazonaws.com/"
        out: Dict[str, float] = {}
        token = None
        for _ in range(20):
            body = json.dumps({"ServiceCode": "ec2", "MaxResults": 100, **({"NextToken": token} if token else {})})
            headers = sigv4_headers("POST", url, region, "servicequotas", self.access_key, self.secret_key,
                                    body.encode(), self.session_token, extra_headers={
                                        "content-type": "application/x-amz-json-1.1",
                                        "x-amz-target": "ServiceQuotasV20190624.ListServiceQuotas"})
            r = self.http.post(url, content=body.encode(), headers=headers)
            if r.status_code >= 400:
                return None
            d = r.json()
            for q in d.get("Quotas") or []:
                cls = ((q.get("UsageMetric") or {}).get("MetricDimensions") or {}).get("Class")
                if cls:
                    out[cls] = float(q.get("Value") or 0)
            token = d.get("NextToken")
            if not token:
                break
        return out

    # ---- helpers ------------------------------------------------------------------------------
    def _image_id(self, region: str, gpu: bool) -> str:
        return self.image_id_and_username(region, gpu)[0]

    def _tag_spec(self, kind: str, base: Dict[str, str]) -> Dict[str, str]:
        """``TagSpecification.1.*`` query params: dstack's tags plus the config's ``tags``."""
        out = {"TagSpecification.1.ResourceType": kind}
        for i, (k, v) in enumerate(merged_tags("aws", base, self.config).items(), 1):
            out[f"TagSpecification.1.Tag.{i}.Key"] = k
            out[f"TagSpecification.1.Tag.{i}.Value"] = str(v)
        return out

    def image_id_and_username(self, region: str, gpu: bool) -> Tuple[str, str]:
        """(AMI, SSH user) for an instance with or without GPUs.

        ``os_images`` configures them per kind: ``{"cpu": {"name", "owner", "user"}, "amd": {...}}``
        (name pattern, owner account or ``self``; a kind left out is not launchable), or the
        older ``{"cpu": {region: ami}, "amd": {...}}`` map. Without ``os_images``: Canonical's Ubuntu
        22.04 (the ROCm driver comes from the shim's host setup). The newest *available* image wins."""
        imgs = self.config.get("os_images") or {}
        key = "amd" if gpu else "cpu"
        if imgs:
            spec = imgs.get(key) or (imgs.get("nvidia") if gpu and "amd" not in imgs else None)
            if not spec:
                logger.warning("%s image not configured in os_images", key)
                raise ComputeResourceNotFoundError(f"no {key} image configured in os_images")
            if "name" not in spec:  # region -> AMI map
                if spec.get(region):
                    return spec[region], self.SSH_USER
                raise ComputeResourceNotFoundError(f"no {key} image configured for {region}")
            name, owner, user = spec["name"], spec.get("owner") or "self", spec.get("user") or self.SSH_USER
        else:
            name, owner, user = "ubuntu/images/hvm-ssd/ubuntu-jammy-22.04-amd64-server-*", UBUNTU_OWNER, self.SSH_USER
        items = self._paginate(region, "DescribeImages", {"Owner.1": owner, "Filter.1.Name": "name",
                                                           "Filter.1.Value.1": name}, "./imagesSet/item")
        avail = [(i.findtext("creationDate") or "", i.findtext("imageId")) for i in items
                 if i.findtext("imageId") and (i.findtext("imageState") or "available") == "available"]
        if not avail:
            logger.warning("image '%s' not found in %s", name, region)
            raise ComputeResourceNotFoundError(f"image '{name}' (owner {owner}) not found in {region}")
        return max(avail)[1], user

    def _vpc_id(self, region: str) -> Optional[str]:
        """``vpc_ids: {region: vpc-...}`` or ``vpc_name`` (tag Name) from the backend config; None =
        the region's default VPC (no explicit subnet)."""
        ids = self.config.get("vpc_ids") or {}
        if isinstance(ids, dict) and ids.get(region):
            return ids[region]
        name = self.config.get("vpc_name")
        if not name:
            return None
        vpcs = self._paginate(region, "DescribeVpcs", {"Filter.1.Name": "tag:Name", "Filter.1.Value.1": name},
                              "./vpcSet/item")
        if not vpcs:
            raise ComputeError(f"no VPC named {name!r} in {region}")
        return vpcs[0].findtext("vpcId")

    def _subnets(self, region: str, vpc_id: Optional[str], public_ip: bool) -> List[Tuple[str, str]]:
        """[(subnet id, availability zone)] to try, in AZ order.  Configured ``subnet_ids`` win; in a
        named VPC public-IP launches use subnets that map public IPs on launch."""
        conf = self.config.get("subnet_ids")
        params: Dict[str, str] = {}
        if isinstance(conf, dict) and conf.get(region):
            sids = conf[region] if isinstance(conf[region], list) else [conf[region]]
            for i, sid in enumerate(sids, 1):
                params[f"SubnetId.{i}"] = sid
        elif vpc_id is not None:
            params = {"Filter.1.Name": "vpc-id", "Filter.1.Value.1": vpc_id}
        else:
            return []
        out = []
        for it in self._paginate(region, "DescribeSubnets", params, "./subnetSet/item"):
            if vpc_id is not None and "SubnetId.1" not in params and public_ip and \
                    (it.findtext("mapPublicIpOnLaunch") or "false") != "true":
                continue
            out.append((it.findtext("subnetId"), it.findtext("availabilityZone") or ""))
        if not out:
            raise ComputeError(f"no usable subnet in {vpc_id or 'the configured subnets'} ({region})")
        return sorted(out, key=lambda x: x[1])

    def _max_efa_interfaces(self, region: str, instance_type: str) -> int:
        """EFA network cards of ``instance_type`` (0 when EFA is not supported); the RDMA NICs RCCL's
        net plugin uses across nodes (reference ``get_maximum_efa_interfaces``)."""
        try:
            items = self._paginate(region, "DescribeInstanceTypes", {"InstanceType.1": instance_type},
                                   "./instanceTypeSet/item")
        except ComputeError:
            return 0
        if not items:
            return 0
        net = items[0].find("networkInfo")
        if net is None or (net.findtext("efaSupported") or "false") != "true":
            return 0
        return int(net.findtext("efaInfo/maximumEfaInterfaces") or net.findtext("maximumNetworkCards") or 1)

    def _reservation(self, region: str, reservation_id: str) -> Dict[str, str]:
        items = self._paginate(region, "DescribeCapacityReservations",
                               {"CapacityReservationId.1": reservation_id}, "./capacityReservationSet/item")
        if not items:
            raise NoCapacityError(f"capacity reservation {reservation_id} not found in {region}")
        it = items[0]
        state = it.findtext("state")
        if state not in ("active", "scheduled"):
            raise NoCapacityError(f"capacity reservation {reservation_id} is {state}")
        return {"az": it.findtext("availabilityZone") or "", "type": it.findtext("reservationType") or "default",
                "instance_type": it.findtext("instanceType") or ""}

    def _security_group(self, region: str, project: str, vpc_id: Optional[str] = None) -> str:
        name = f"dstack_{project}"
        params = {"Filter.1.Name": "group-name", "Filter.1.Value.1": name}
        if vpc_id:
            params.update({"Filter.2.Name": "vpc-id", "Filter.2.Value.1": vpc_id})
        root = self._call(region, "DescribeSecurityGroups", params)
        gid = root.findtext(".//securityGroupInfo/item/groupId")
        if gid:
            return gid
        create = {"GroupName": name, "GroupDescription": "dstack-amd"}
        if vpc_id:
            create["VpcId"] = vpc_id
        root = self._call(region, "CreateSecurityGroup", create)
        gid = root.findtext("groupId")
        self._call(region, "AuthorizeSecurityGroupIngress", {
            "GroupId": gid, "IpPermissions.1.IpProtocol": "tcp", "IpPermissions.1.FromPort": "22",
            "IpPermissions.1.ToPort": "22", "IpPermissions.1.IpRanges.1.CidrIp": "0.0.0.0/0"})
        # intra-cluster traffic (RCCL/torchrun between nodes of a fleet, EFA needs all-to-all in SG)
        self._call(region, "AuthorizeSecurityGroupIngress", {
            "GroupId": gid, "IpPermissions.1.IpProtocol": "-1",
            "IpPermissions.1.Groups.1.GroupId": gid})
        return gid

    # ---- VMCompute hooks ----------------------------------------------------------------------
    def _run_params(self, offer: InstanceOfferWithAvailability, cfg: InstanceConfiguration, image_id: str,
                    sg: str, subnet: Optional[str], efa: int, public_ip: bool, capacity_block: bool) -> Dict[str, str]:
        res = offer.instance.resources
        params = {
            "ImageId": image_id, "InstanceType": offer.instance.name, "MinCount": "1", "MaxCount": "1",
            "UserData": base64.b64encode(cloud_init(cfg).encode()).decode(),
            "BlockDeviceMapping.1.DeviceName": "/dev/sda1",
            "BlockDeviceMapping.1.Ebs.VolumeSize": str(max(100, res.disk.size_mib // 1024)),
            "BlockDeviceMapping.1.Ebs.VolumeType": "gp3",
            **self._tag_spec("instance", {"Name": cfg.instance_name, "owner": "dstack",
                                          "dstack_project": cfg.project_name, "dstack_user": cfg.user or ""}),
        }
        if capacity_block:
            params["InstanceMarketOptions.MarketType"] = "capacity-block"
        elif res.spot:
            params["InstanceMarketOptions.MarketType"] = "spot"
            params["InstanceMarketOptions.SpotOptions.SpotInstanceType"] = "one-time"
            params["InstanceMarketOptions.SpotOptions.InstanceInterruptionBehavior"] = "terminate"
        if cfg.placement_group_name:
            params["Placement.GroupName"] = cfg.placement_group_name
        if cfg.reservation:
            params["CapacityReservationSpecification.CapacityReservationTarget.CapacityReservationId"] = \
                cfg.reservation
        if subnet is None:
            params["SecurityGroupId.1"] = sg  # default VPC: instance-level security group
            return params
        # an explicit subnet: interfaces carry subnet + security group (AWS takes one or the other);
        # EFA cards beyond the first only without a public IP (one interface may associate it)
        nics = [{"DeviceIndex": "0", "SubnetId": subnet, "SecurityGroupId.1": sg,
                 "AssociatePublicIpAddress": "true" if public_ip else "false",
                 "InterfaceType": "efa" if efa > 0 else "interface"}]
        if efa > 1 and not public_ip:
            for card in range(1, efa):
                # p5: every 4th card keeps the IP stack (efa), the rest are RDMA-only (efa-only)
                kind = "efa" if offer.instance.name.startswith("p5") and card % 4 == 0 else "efa-only"
                nics.append({"NetworkCardIndex": str(card), "DeviceIndex": "1", "SubnetId": subnet,
                             "SecurityGroupId.1": sg, "AssociatePublicIpAddress": "false", "InterfaceType": kind})
        for n, nic in enumerate(nics, 1):
            for k, v in nic.items():
                params[f"NetworkInterface.{n}.{k}"] = v
        return params

    def _launch(self, offer: InstanceOfferWithAvailability, cfg: InstanceConfiguration
                ) -> Tuple[str, Optional[str], Optional[dict]]:
        region = offer.region
        public_ip = bool(self.config.get("public_ips", True))
        vpc_id = self._vpc_id(region)
        subnets: List[Tuple[Optional[str], str]] = list(self._subnets(region, vpc_id, public_ip))
        efa = self._max_efa_interfaces(region, offer.instance.name) if subnets else 0
        capacity_block = False
        if cfg.reservation:
            rsv = self._reservation(region, cfg.reservation)
            capacity_block = rsv["type"] == "capacity-block"
            if subnets:
                subnets = [x for x in subnets if x[1] == rsv["az"]]
                if not subnets:
                    raise NoCapacityError(f"no subnet in the reservation's zone {rsv['az']}")
            elif not cfg.availability_zone:
                cfg = cfg.model_copy(update={"availability_zone": rsv["az"]})
        if cfg.availability_zone and subnets:
            subnets = [x for x in subnets if x[1] == cfg.availability_zone] or subnets
        image_id, ssh_user = self.image_id_and_username(region, bool(offer.instance.resources.gpus))
        sg = self._security_group(region, cfg.project_name, vpc_id)
        attempts = subnets or [(None, cfg.availability_zone or "")]
        tried, last = set(), None
        for subnet, az in attempts:
            if az in tried:
                continue  # one try per zone
            tried.add(az)
            params = self._run_params(offer, cfg, image_id, sg, subnet, efa, public_ip, capacity_block)
            if subnet is None and az:
                params["Placement.AvailabilityZone"] = az
            try:
                root = self._call(region, "RunInstances", params)
            except NoCapacityError as e:
                last = e
                continue
            iid = root.findtext(".//instancesSet/item/instanceId")
            if not iid:
                raise ComputeError("RunInstances returned no instance id")
            return iid, None, {"region": region, "public_ip": public_ip, "efa_interfaces": efa, "ssh_user": ssh_user}
        raise last or NoCapacityError(f"no capacity for {offer.instance.name} in {region}")

    def _describe(self, instance_id: str, region: str, backend_data: dict) -> dict:
        root = self._call(region, "DescribeInstances", {"InstanceId.1": instance_id})
        item = root.find(".//instancesSet/item")
        if item is None:
            return {"status": "pending"}
        state = item.findtext("instanceState/name")
        if state in ("terminated", "shutting-down"):
            return {"status": "terminated"}
        if backend_data.get("public_ip") is False:  # private subnets: reach it on its VPC address
            return {"status": state, "hostname": item.findtext("privateIpAddress") if state == "running" else None,
                    "internal_ip": item.findtext("privateIpAddress")}
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
            **self._tag_spec("volume", {"Name": volume.name, "owner": "dstack",
                                        "dstack_project": volume.project_name})})
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
        """A small VM running the gateway package.  ``public_ip: false`` (private gateway): it is
        launched into the configured VPC's subnets without a public address and served on its
        private IP (reachable from inside the VPC, e.g. behind an internal load balancer)."""
        import time

        from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init

        region = configuration.region
        public = configuration.public_ip
        sg = self._gateway_security_group(region, configuration.project_name, self._vpc_id(region))
        params = {"ImageId": self._image_id(region, False), "InstanceType": "t3.small", "MinCount": "1",
                  "MaxCount": "1", "UserData": base64.b64encode(gateway_cloud_init(configuration).encode()).decode(),
                  **self._tag_spec("instance", {"Name": configuration.instance_name, "owner": "dstack",
                                                "dstack_project": configuration.project_name, "role": "gateway"})}
        subnets = self._subnets(region, self._vpc_id(region), public)
        if subnets or not public:
            if not subnets:
                raise ComputeError(f"a private gateway needs vpc_name / vpc_ids / subnet_ids for {region}")
            params.update({"NetworkInterface.1.DeviceIndex": "0", "NetworkInterface.1.SubnetId": subnets[0][0],
                           "NetworkInterface.1.AssociatePublicIpAddress": "true" if public else "false",
                           "NetworkInterface.1.SecurityGroupId.1": sg})
        else:
            params["SecurityGroupId.1"] = sg
        root = self._call(region, "RunInstances", params)
        iid = root.findtext(".//instancesSet/item/instanceId")
        ip = None
        for _ in range(60):
            info = self._describe(iid, region, {"public_ip": public})
            if info.get("hostname"):
                ip = info["hostname"]
                break
            time.sleep(float(self.config.get("gateway_poll_s", 5)))
        if ip is None:
            raise ComputeError(f"gateway {iid} got no {'public' if public else 'private'} IP")
        return GatewayProvisioningData(instance_id=iid, ip_address=ip, region=region,
                                       backend_data=json.dumps({"public_ip": public}))

    def _gateway_security_group(self, region: str, project: str, vpc_id: Optional[str] = None) -> str:
        gid = self._security_group(region, f"{project}_gateway", vpc_id)
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

