"""Azure, GCP and OCI over their REST APIs (reference: ``C/backends/azure/compute.py`` (839 LoC,
azure-mgmt SDK), ``C/backends/gcp/compute.py`` (1378, google-cloud SDK), ``C/backends/oci/compute.py``
(1181, oci SDK)).

* Azure: OAuth2 client credentials -> one ARM template deployment per VM (project NSG + VNet
  ``dstack-vnet-<region>`` declared idempotently, public IP + NIC + VM with cloud-init
  ``customData``); the MI300X path is ``Standard_ND96isr_MI300X_v5``.  Gateways: a small VM with its
  own NSG (22/80/443).
* GCP: service-account JWT (RS256 via OpenSSL) -> ``instances.insert`` with a NAT access config;
  gateways (firewall rule on the ``dstack-gateway`` tag) and zonal persistent-disk volumes
  (create / register / attach / detach / delete, operations awaited).
* OCI: HTTP-signature auth (RSA-SHA256 via OpenSSL) -> ``LaunchInstance`` with the newest
  shape-compatible Ubuntu 22.04 image unless one is configured; the ``BM.GPU.MI300X.8`` bare-metal
  shape takes up to 20 minutes to boot (the reference's 1200 s timeout).
"""

from __future__ import annotations

import base64
import email.utils
import enum
import hashlib
import json
import re
import time
import urllib.parse
from dataclasses import dataclass, replace
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.backends.catalog import CatalogRow, offline_rows
from dstack_amd.core.backends.clouds.tags import merged_tags
from dstack_amd.core.backends.clouds.common import (
    OAuthToken,
    VMCompute,
    b64url,
    check_response,
    cloud_init,
    rsa_sha256_sign,
)
from dstack_amd.core.errors import BackendAuthError, ComputeError, ServerClientError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceAvailability, InstanceType


class AzureImageVariant(enum.Enum):
    """Which marketplace image an Azure VM boots (the reference picks among its own prebuilt
    ``dstack-{,cuda-,grid-}<ver>`` images, ``C/backends/azure/compute.py:342-363``; here the vendor
    images are used and the shim installs the rest):

    * ``ROCM``: AMD Instinct VMs (``ND*_MI300X_v5``) -> the HPC image with ROCm and the amdgpu driver.
    * ``NVIDIA``: NVIDIA VMs -> the HPC image with the CUDA driver (``_A10_v5`` GRID VMs included;
      they need the GRID driver, which the shim's host setup installs).
    * ``STANDARD``: CPU VMs -> Canonical Ubuntu 22.04.

    ``vm_images`` in the backend config overrides any of them by variant name in lower case
    (``{"rocm": {"publisher", "offer", "sku", "version"}}``)."""

    ROCM = "rocm"
    NVIDIA = "nvidia"
    STANDARD = "standard"

    @classmethod
    def from_instance_type(cls, instance: InstanceType) -> "AzureImageVariant":
        gpus = instance.resources.gpus
        if not gpus:
            return cls.STANDARD
        g = gpus[0]
        vendor = getattr(g.vendor, "value", g.vendor)
        if vendor == "amd" or "MI300X" in instance.name or g.name.upper().startswith("MI"):
            return cls.ROCM
        return cls.NVIDIA

    def image_reference(self, overrides: Optional[dict] = None) -> dict:
        over = (overrides or {}).get(self.value)
        if over:
            return {"version": "latest", **over}
        return {
            AzureImageVariant.ROCM: {"publisher": "microsoft-dsvm", "offer": "ubuntu-hpc", "sku": "2204-rocm",
                                     "version": "latest"},
            AzureImageVariant.NVIDIA: {"publisher": "microsoft-dsvm", "offer": "ubuntu-hpc", "sku": "2204",
                                       "version": "latest"},
            AzureImageVariant.STANDARD: {"publisher": "Canonical", "offer": "0001-com-ubuntu-server-jammy",
                                         "sku": "22_04-lts-gen2", "version": "latest"},
        }[self]


def gcp_label(value: str) -> str:
    """A GCP label value from a free-form name: lower case, ``[a-z0-9_-]``, at most 63 characters."""
    return re.sub(r"[^a-z0-9_\-]", "-", value.lower())[:63]


# ---------------------------------------------------------------------------------------------
class AzureCompute(VMCompute):
    TYPE = BackendType.AZURE
    ARM = "https://management.azure.com"
    SSH_USER = "ubuntu"

    def __init__(self, config, auth, client=None):
        super().__init__(config, auth, client)
        self._token = OAuthToken(self._fetch_token)
        self.subscription = self.config.get("subscription_id") or self.auth.get("subscription_id")
        self.tenant = self.config.get("tenant_id") or self.auth.get("tenant_id")

    def _fetch_token(self):
        r = self.http.post(
            f"https://login.microsoftonline.com/{self.tenant}/oauth2/v2.0/token",
            data={"grant_type": "client_credentials", "client_id": self.auth.get("client_id"),
                  "client_secret": self.auth.get("client_secret"), "scope": f"{self.ARM}/.default"})
        if r.status_code in (400, 401):  # AADSTS errors: unknown tenant / client, bad secret
            raise BackendAuthError(f"azure token: {r.status_code} {r.text[:300]}")
        d = check_response(r, "azure token").json()
        return d["access_token"], d.get("expires_in", 3600)

    def _h(self):
        return {"Authorization": f"Bearer {self._token.get()}"}

    CONFIGURABLE_DISK = (30.0, 4095.0)  # managed OS disk, GiB

    def check_credentials(self) -> None:
        """Token exchange + read access to the subscription."""
        r = self.http.get(f"{self.ARM}/subscriptions/{self.subscription}?api-version=2020-01-01", headers=self._h())
        if r.status_code in (401, 403, 404):
            raise BackendAuthError(f"azure subscription {self.subscription}: {r.status_code} {r.text[:200]}")
        check_response(r, "azure subscription")
    RETAIL_PRICES = "https://prices.azure.com/api/retail/prices"

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Catalog SKUs priced from the public Retail Prices API (Linux pay-as-you-go and Spot
        meters, every region that sells them) and checked against the subscription's resource-SKU
        restrictions (``NotAvailableForSubscription`` -> ``no_quota``)."""
        base = offline_rows(self.TYPE)
        specs: Dict[str, CatalogRow] = {}
        for r in base:
            specs.setdefault(r.instance_name, r)
        prices = self._retail_prices(sorted(specs))
        wanted = self.regions()
        restricted = self._restricted_skus() if self.subscription else {}
        out = []
        for (sku, region, spot), price in sorted(prices.items()):
            if wanted and region not in wanted:
                continue
            avail = InstanceAvailability.NO_QUOTA if region in restricted.get(sku, ()) else InstanceAvailability.UNKNOWN
            out.append(replace(specs[sku], location=region, spot=spot, price=round(price, 6), availability=avail))
        return out

    def _retail_prices(self, skus: List[str]) -> Dict[Tuple[str, str, bool], float]:
        flt = "serviceName eq 'Virtual Machines' and priceType eq 'Consumption' and (" + \
            " or ".join(f"armSkuName eq '{s}'" for s in skus) + ")"
        url: Optional[str] = f"{self.RETAIL_PRICES}?{urllib.parse.urlencode({'$filter': flt})}"
        out: Dict[Tuple[str, str, bool], float] = {}
        for _ in range(50):
            if not url:
                break
            d = check_response(self.http.get(url), "azure retail prices").json()
            for it in d.get("Items") or []:
                name = it.get("skuName") or ""
                if "Windows" in (it.get("productName") or "") or "Low Priority" in name:
                    continue
                if it.get("unitOfMeasure", "1 Hour") != "1 Hour":
                    continue
                key = (it.get("armSkuName"), it.get("armRegionName"), "Spot" in name)
                price = float(it.get("retailPrice") or 0)
                if price > 0:
                    out[key] = min(price, out.get(key, price))
            url = d.get("NextPageLink")
        return out

    def _restricted_skus(self) -> Dict[str, set]:
        url = (f"{self.ARM}/subscriptions/{self.subscription}/providers/Microsoft.Compute/skus"
               "?api-version=2021-07-01")
        out: Dict[str, set] = {}
        for _ in range(50):
            d = check_response(self.http.get(url, headers=self._h()), "azure resource skus").json()
            for sku in d.get("value") or []:
                if sku.get("resourceType") != "virtualMachines":
                    continue
                for rs in sku.get("restrictions") or []:
                    if rs.get("reasonCode") == "NotAvailableForSubscription" and rs.get("type") == "Location":
                        locs = (rs.get("restrictionInfo") or {}).get("locations") or rs.get("values") or []
                        out.setdefault(sku.get("name"), set()).update(l.lower() for l in locs)
            url = d.get("nextLink")
            if not url:
                break
        return out

    def _rg(self, region: str) -> str:
        rg = (self.config.get("resource_groups") or {}).get(region) or f"dstack-{region}"
        url = f"{self.ARM}/subscriptions/{self.subscription}/resourcegroups/{rg}?api-version=2021-04-01"
        check_response(self.http.put(url, headers=self._h(), json={"location": region}), "azure resource group")
        return rg

    @staticmethod
    def _rule(name: str, prio: int, port: str) -> dict:
        return {"name": name, "properties": {"priority": prio, "direction": "Inbound", "access": "Allow",
                                             "protocol": "Tcp", "sourcePortRange": "*", "destinationPortRange": port,
                                             "sourceAddressPrefix": "*", "destinationAddressPrefix": "*"}}

    def _network_resources(self, region: str) -> list:
        """The project network every VM of the region joins, declared in each deployment
        (idempotent in Incremental mode): an NSG admitting SSH plus all traffic inside the VNet
        (RCCL/torchrun between nodes), and ``dstack-vnet-<region>`` with subnet ``default``."""
        nsg = f"dstack-nsg-{region}"
        rules = [self._rule("ssh", 100, "22"),
                 {"name": "vnet", "properties": {"priority": 110, "direction": "Inbound", "access": "Allow",
                                                 "protocol": "*", "sourcePortRange": "*", "destinationPortRange": "*",
                                                 "sourceAddressPrefix": "VirtualNetwork",
                                                 "destinationAddressPrefix": "VirtualNetwork"}}]
        return [
            {"type": "Microsoft.Network/networkSecurityGroups", "apiVersion": "2023-04-01", "name": nsg,
             "location": region, "properties": {"securityRules": rules}},
            {"type": "Microsoft.Network/virtualNetworks", "apiVersion": "2023-04-01", "name": f"dstack-vnet-{region}",
             "location": region, "dependsOn": [f"[resourceId('Microsoft.Network/networkSecurityGroups', '{nsg}')]"],
             "properties": {"addressSpace": {"addressPrefixes": ["10.0.0.0/16"]}, "subnets": [
                 {"name": "default", "properties": {"addressPrefix": "10.0.0.0/20", "networkSecurityGroup": {
                     "id": f"[resourceId('Microsoft.Network/networkSecurityGroups', '{nsg}')]"}}}]}},
        ]

    def _template(self, name: str, size: str, region: str, user_data: str, disk_gb: int, spot: bool,
                  public_keys, extra_ports=(), image: Optional[dict] = None, tags: Optional[dict] = None) -> dict:
        own_network = not self.config.get("subnet_id")
        subnet = self.config.get("subnet_id") or (
            f"[resourceId('Microsoft.Network/virtualNetworks/subnets', 'dstack-vnet-{region}', 'default')]")
        vm_props = {
            "hardwareProfile": {"vmSize": size},
            "storageProfile": {"imageReference": image or AzureImageVariant.STANDARD.image_reference(
                                   self.config.get("vm_images")),
                               "osDisk": {"createOption": "FromImage", "diskSizeGB": disk_gb,
                                          "deleteOption": "Delete"}},
            "osProfile": {"computerName": name[:15], "adminUsername": self.SSH_USER,
                          "customData": base64.b64encode(user_data.encode()).decode(),
                          "linuxConfiguration": {"disablePasswordAuthentication": True, "ssh": {"publicKeys": [
                              {"path": f"/home/{self.SSH_USER}/.ssh/authorized_keys", "keyData": k}
                              for k in public_keys]}}},
            "networkProfile": {"networkInterfaces": [{"id": f"[resourceId('Microsoft.Network/networkInterfaces', "
                                                            f"'{name}-nic')]",
                                                      "properties": {"deleteOption": "Delete"}}]},
        }
        if spot:
            vm_props.update({"priority": "Spot", "evictionPolicy": "Delete", "billingProfile": {"maxPrice": -1}})
        nic_deps = [f"[resourceId('Microsoft.Network/publicIPAddresses', '{name}-ip')]"]
        res = self._network_resources(region) if own_network else []
        if own_network:
            nic_deps.append(f"[resourceId('Microsoft.Network/virtualNetworks', 'dstack-vnet-{region}')]")
        nic_props = {"enableAcceleratedNetworking": True, "ipConfigurations": [{"name": "ipconfig1", "properties": {
            "subnet": {"id": subnet}, "publicIPAddress": {"id": f"[resourceId('Microsoft.Network/"
                                                                  f"publicIPAddresses', '{name}-ip')]"}}}]}
        if extra_ports:  # a gateway: its own NSG on the NIC admits HTTP(S) from anywhere
            gnsg = f"{name}-nsg"
            res.append({"type": "Microsoft.Network/networkSecurityGroups", "apiVersion": "2023-04-01", "name": gnsg,
                        "location": region, "properties": {"securityRules": [
                            self._rule(f"p{p}", 100 + i, str(p)) for i, p in enumerate((22, *extra_ports))]}})
            nic_deps.append(f"[resourceId('Microsoft.Network/networkSecurityGroups', '{gnsg}')]")
            nic_props["networkSecurityGroup"] = {"id": f"[resourceId('Microsoft.Network/networkSecurityGroups', "
                                                       f"'{gnsg}')]"}
            nic_props["enableAcceleratedNetworking"] = False
        res += [
            {"type": "Microsoft.Network/publicIPAddresses", "apiVersion": "2023-04-01", "name": f"{name}-ip",
             "location": region, "sku": {"name": "Standard"}, "properties": {"publicIPAllocationMethod": "Static"}},
            {"type": "Microsoft.Network/networkInterfaces", "apiVersion": "2023-04-01", "name": f"{name}-nic",
             "location": region, "dependsOn": nic_deps, "properties": nic_props},
            {"type": "Microsoft.Compute/virtualMachines", "apiVersion": "2023-03-01", "name": name, "location": region,
             "dependsOn": [f"[resourceId('Microsoft.Network/networkInterfaces', '{name}-nic')]"],
             "properties": vm_props},
        ]
        tags = merged_tags("azure", {"owner": "dstack", **(tags or {})}, self.config)
        for r in res:
            r["tags"] = tags
        return {"$schema": "https://schema.management.azure.com/schemas/2019-04-01/deploymentTemplate.json#",
                "contentVersion": "1.0.0.0", "resources": res}

    def _launch(self, offer, cfg):
        region = offer.region
        rg = self._rg(region)
        name = cfg.instance_name.replace("_", "-")[:60]
        image = AzureImageVariant.from_instance_type(offer.instance).image_reference(self.config.get("vm_images"))
        tpl = self._template(name, offer.instance.name, region, cloud_init(cfg),
                             max(100, offer.instance.resources.disk.size_mib // 1024), offer.instance.resources.spot,
                             cfg.get_public_keys(), image=image,
                             tags={"dstack_project": cfg.project_name, "dstack_user": cfg.user or ""})
        url = (f"{self.ARM}/subscriptions/{self.subscription}/resourcegroups/{rg}/providers/"
               f"Microsoft.Resources/deployments/{name}?api-version=2021-04-01")
        check_response(self.http.put(url, headers=self._h(), json={"properties": {"mode": "Incremental",
                                                                                  "template": tpl}}), "azure deploy")
        return name, None, {"resource_group": rg}

    def _describe(self, instance_id, region, backend_data):
        rg = backend_data.get("resource_group", f"dstack-{region}")
        base = f"{self.ARM}/subscriptions/{self.subscription}/resourceGroups/{rg}/providers"
        dep = self.http.get(f"{base}/Microsoft.Resources/deployments/{instance_id}?api-version=2021-04-01",
                            headers=self._h())
        if dep.status_code == 200 and dep.json().get("properties", {}).get("provisioningState") == "Failed":
            return {"status": "failed", "error": dep.json()["properties"].get("error")}
        ip = self.http.get(f"{base}/Microsoft.Network/publicIPAddresses/{instance_id}-ip?api-version=2023-04-01",
                           headers=self._h())
        if ip.status_code != 200:
            return {"status": "provisioning"}
        addr = ip.json().get("properties", {}).get("ipAddress")
        return {"status": "running" if addr else "provisioning", "hostname": addr}

    def _terminate(self, instance_id, region, backend_data):
        rg = backend_data.get("resource_group", f"dstack-{region}")
        base = f"{self.ARM}/subscriptions/{self.subscription}/resourceGroups/{rg}/providers"
        # the VM deletes its OS disk and NIC (deleteOption); the public IP and a gateway's NSG go
        # after it (Azure refuses to delete an IP still bound to a NIC: the VM delete is awaited)
        paths = [(f"Microsoft.Compute/virtualMachines/{instance_id}", "2023-03-01"),
                 (f"Microsoft.Network/publicIPAddresses/{instance_id}-ip", "2023-04-01")]
        if backend_data.get("gateway"):
            paths.append((f"Microsoft.Network/networkSecurityGroups/{instance_id}-nsg", "2023-04-01"))
        for i, (path, ver) in enumerate(paths):
            r = self.http.delete(f"{base}/{path}?api-version={ver}", headers=self._h())
            if r.status_code not in (200, 202, 204, 404):
                check_response(r, f"azure delete {path}")
            if i == 0 and r.status_code == 202 and r.headers.get("azure-asyncoperation"):
                self._await(r.headers["azure-asyncoperation"])

    def _await(self, op_url: str, tries: int = 120, delay: float = 5.0):
        for _ in range(tries):
            st = self.http.get(op_url, headers=self._h()).json().get("status", "")
            if st in ("Succeeded", "Failed", "Canceled"):
                return st
            time.sleep(delay)
        return "Timeout"

    # ---- gateway ------------------------------------------------------------------------------
    def create_gateway(self, configuration):
        """A small VM (``Standard_B2s``) with the versioned gateway app, its own NSG admitting
        22/80/443, and a static public IP (reference ``C/backends/azure/compute.py`` create_gateway)."""
        from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init
        from dstack_amd.core.models.gateways import GatewayProvisioningData

        region = configuration.region
        rg = self._rg(region)
        name = f"{configuration.instance_name}".replace("_", "-")[:60]
        tpl = self._template(name, self.config.get("gateway_vm_size", "Standard_B2s"), region,
                             gateway_cloud_init(configuration), 30, False, [configuration.ssh_key_pub.strip()],
                             extra_ports=(80, 443), tags={"dstack_project": configuration.project_name,
                                                          "role": "gateway"})
        url = (f"{self.ARM}/subscriptions/{self.subscription}/resourcegroups/{rg}/providers/"
               f"Microsoft.Resources/deployments/{name}?api-version=2021-04-01")
        check_response(self.http.put(url, headers=self._h(), json={"properties": {"mode": "Incremental",
                                                                                  "template": tpl}}), "azure gateway")
        data = {"resource_group": rg, "gateway": True}
        for _ in range(120):
            info = self._describe(name, region, data)
            if info.get("status") == "failed":
                raise ComputeError(f"azure gateway deployment failed: {info.get('error')}")
            if info.get("hostname"):
                return GatewayProvisioningData(instance_id=name, ip_address=info["hostname"], region=region,
                                               backend_data=json.dumps(data))
            time.sleep(5)
        raise ComputeError(f"azure gateway {name} got no public IP")

    def terminate_gateway(self, instance_id, configuration, backend_data=None):
        data = json.loads(backend_data or "{}")
        data.setdefault("gateway", True)
        self._terminate(instance_id, configuration.region, data)


# ---------------------------------------------------------------------------------------------
class GCPCompute(VMCompute):
    TYPE = BackendType.GCP
    API = "https://compute.googleapis.com/compute/v1"
    SSH_USER = "ubuntu"

    def __init__(self, config, auth, client=None):
        super().__init__(config, auth, client)
        sa = self.auth.get("data") or self.auth
        self.sa = json.loads(sa) if isinstance(sa, str) else sa
        self.project = self.config.get("project_id") or self.sa.get("project_id")
        self._token = OAuthToken(self._fetch_token)

    def _fetch_token(self):
        now = int(time.time())
        header = b64url(json.dumps({"alg": "RS256", "typ": "JWT"}).encode())
        claims = b64url(json.dumps({"iss": self.sa["client_email"], "scope": "https://www.googleapis.com/auth/cloud-platform",
                                    "aud": "https://oauth2.googleapis.com/token", "iat": now, "exp": now + 3600}).encode())
        sig = b64url(rsa_sha256_sign(self.sa["private_key"], f"{header}.{claims}".encode()))
        r = self.http.post("https://oauth2.googleapis.com/token", data={
            "grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer", "assertion": f"{header}.{claims}.{sig}"})
        if r.status_code in (400, 401):  # invalid_grant: unknown / disabled key
            raise BackendAuthError(f"gcp token: {r.status_code} {r.text[:300]}")
        d = check_response(r, "gcp token").json()
        return d["access_token"], d.get("expires_in", 3600)

    def _h(self):
        return {"Authorization": f"Bearer {self._token.get()}"}

    CONFIGURABLE_DISK = (10.0, 65536.0)  # persistent boot disk, GB

    def check_credentials(self) -> None:
        """Token exchange + the Compute API on the project (403 / 404: no access or no API)."""
        if not self.sa.get("client_email") or not self.sa.get("private_key"):
            raise BackendAuthError("gcp: the service-account key needs client_email and private_key")
        r = self.http.get(f"{self.API}/projects/{self.project}", headers=self._h())
        if r.status_code in (401, 403, 404):
            raise BackendAuthError(f"gcp project {self.project}: {r.status_code} {r.text[:200]}")
        check_response(r, "gcp project")

    def _machine_type_zones(self, names) -> Dict[Tuple[str, str], List[str]]:
        """{(machine type, region): [zones offering it]} from the aggregated machineTypes list."""
        flt = " OR ".join(f'(name = "{n}")' for n in sorted(names))
        zones: Dict[Tuple[str, str], List[str]] = {}
        token = None
        for _ in range(50):
            params = {"filter": flt, "maxResults": 500, **({"pageToken": token} if token else {})}
            d = check_response(self.http.get(f"{self.API}/projects/{self.project}/aggregated/machineTypes",
                                             params=params, headers=self._h()), "gcp machine types").json()
            for scope, v in (d.get("items") or {}).items():
                zone = scope.split("/", 1)[-1]
                region = zone.rsplit("-", 1)[0]
                for mt in v.get("machineTypes") or []:
                    zones.setdefault((mt.get("name"), region), []).append(zone)
            token = d.get("nextPageToken")
            if not token:
                break
        return {k: sorted(v) for k, v in zones.items()}

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Catalog machine types checked against the project's zones (aggregated
        ``machineTypes`` list): regions where a type is offered in some zone keep the catalog
        price (``unknown`` stock), the rest are ``not_available``; zones offering each type are
        remembered for the launch."""
        base = offline_rows(self.TYPE)
        zones = self._machine_type_zones({r.instance_name for r in base})
        self._type_zones = zones
        out = []
        wanted = self.config.get("regions")
        specs: Dict[str, List[CatalogRow]] = {}
        for r in base:
            specs.setdefault(r.instance_name, []).append(r)
        for name, rows in specs.items():
            offered = {reg for (n, reg) in zones if n == name}
            for spot in sorted({r.spot for r in rows}):
                proto = next(r for r in rows if r.spot == spot)
                for region in sorted(offered | {r.location for r in rows if r.spot == spot}):
                    if wanted and region not in wanted:
                        continue
                    out.append(replace(proto, location=region, availability=InstanceAvailability.UNKNOWN
                                       if region in offered else InstanceAvailability.NOT_AVAILABLE))
        return out

    def _zone(self, region: str, machine_type: Optional[str] = None) -> str:
        zones = self.config.get("zones") or {}
        if zones.get(region):
            return zones[region]
        if not machine_type:
            return f"{region}-a"
        known = getattr(self, "_type_zones", None)
        if known is None or (machine_type, region) not in known:
            # offers served from the catalog cache (another process, or no live listing): ask once
            try:
                found = self._machine_type_zones({machine_type})
            except Exception:  # noqa: BLE001 -- keep the conventional first zone
                found = {}
            self._type_zones = {**(known or {}), **found}
        offered = self._type_zones.get((machine_type, region))
        return offered[0] if offered else f"{region}-a"

    def _launch(self, offer, cfg):
        zone = self._zone(offer.region, offer.instance.name)
        res = offer.instance.resources
        name = cfg.instance_name.lower().replace("_", "-")[:62]
        body = {
            "name": name, "machineType": f"zones/{zone}/machineTypes/{offer.instance.name}",
            "disks": [{"boot": True, "autoDelete": True, "initializeParams": {
                "sourceImage": "projects/ubuntu-os-cloud/global/images/family/ubuntu-2204-lts",
                "diskSizeGb": str(max(100, res.disk.size_mib // 1024)), "diskType": f"zones/{zone}/diskTypes/pd-balanced"}}],
            "networkInterfaces": [{"network": self.config.get("vpc", "global/networks/default"),
                                   "accessConfigs": [{"type": "ONE_TO_ONE_NAT", "name": "External NAT"}]}],
            "metadata": {"items": [{"key": "user-data", "value": cloud_init(cfg)},
                                   {"key": "ssh-keys", "value": "\n".join(f"{self.SSH_USER}:{k}"
                                                                         for k in cfg.get_public_keys())}]},
            "labels": merged_tags("gcp", {"owner": "dstack", "dstack_project": gcp_label(cfg.project_name),
                                          "dstack_user": gcp_label(cfg.user or "")}, self.config),
            "scheduling": {"provisioningModel": "SPOT" if res.spot else "STANDARD",
                           "onHostMaintenance": "TERMINATE" if res.gpus else "MIGRATE",
                           "automaticRestart": False},
        }
        url = f"{self.API}/projects/{self.project}/zones/{zone}/instances"
        check_response(self.http.post(url, headers=self._h(), json=body), "gcp insert")
        return name, None, {"zone": zone}

    def _describe(self, instance_id, region, backend_data):
        zone = backend_data.get("zone", self._zone(region))
        r = self.http.get(f"{self.API}/projects/{self.project}/zones/{zone}/instances/{instance_id}", headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        d = check_response(r, "gcp get").json()
        nic = (d.get("networkInterfaces") or [{}])[0]
        nat = ((nic.get("accessConfigs") or [{}])[0]).get("natIP")
        st = d.get("status", "").lower()
        return {"status": st, "hostname": nat if st == "running" else None, "internal_ip": nic.get("networkIP")}

    def _terminate(self, instance_id, region, backend_data):
        zone = backend_data.get("zone", self._zone(region))
        r = self.http.delete(f"{self.API}/projects/{self.project}/zones/{zone}/instances/{instance_id}",
                             headers=self._h())
        if r.status_code != 404:
            check_response(r, "gcp delete")

    def _wait_op(self, r, what: str, tries: int = 120, delay: float = 2.0) -> dict:
        """Wait for a zonal/global operation returned by a mutating call; raise on its error."""
        op = r.json()
        link = op.get("selfLink")
        for _ in range(tries):
            if op.get("status") == "DONE":
                if op.get("error"):
                    errs = op["error"].get("errors") or [{}]
                    msg = "; ".join(f"{e.get('code')}: {e.get('message')}" for e in errs)
                    from dstack_amd.core.errors import NoCapacityError

                    if any("RESOURCE" in (e.get("code") or "") or "STOCKOUT" in (e.get("code") or "") for e in errs):
                        raise NoCapacityError(f"{what}: {msg}")
                    raise ComputeError(f"{what}: {msg}")
                return op
            if not link:
                return op
            time.sleep(delay)
            op = check_response(self.http.get(link, headers=self._h()), what).json()
        raise ComputeError(f"{what}: operation did not finish")

    # ---- gateway ------------------------------------------------------------------------------
    GATEWAY_TAG = "dstack-gateway"

    def _gateway_firewall(self):
        body = {"name": "dstack-gateway-in-all", "network": self.config.get("vpc", "global/networks/default"),
                "direction": "INGRESS", "targetTags": [self.GATEWAY_TAG], "sourceRanges": ["0.0.0.0/0"],
                "allowed": [{"IPProtocol": "tcp", "ports": ["22", "80", "443"]}],
                "description": "dstack-amd gateways: SSH from the server, HTTP(S) from clients"}
        r = self.http.post(f"{self.API}/projects/{self.project}/global/firewalls", headers=self._h(), json=body)
        if r.status_code != 409:  # already exists
            self._wait_op(check_response(r, "gcp gateway firewall"), "gcp gateway firewall")

    def create_gateway(self, configuration):
        """An ``e2-small`` VM tagged ``dstack-gateway`` (firewall 22/80/443) running the versioned
        gateway app; waits for its external IP (reference ``C/backends/gcp/compute.py``)."""
        from dstack_amd.core.backends.clouds.gateway_boot import gateway_cloud_init
        from dstack_amd.core.models.gateways import GatewayProvisioningData

        self._gateway_firewall()
        zone = self._zone(configuration.region)
        name = configuration.instance_name.lower().replace("_", "-")[:62]
        body = {
            "name": name, "machineType": f"zones/{zone}/machineTypes/{self.config.get('gateway_machine_type', 'e2-small')}",
            "tags": {"items": [self.GATEWAY_TAG]},
            "disks": [{"boot": True, "autoDelete": True, "initializeParams": {
                "sourceImage": "projects/ubuntu-os-cloud/global/images/family/ubuntu-2204-lts", "diskSizeGb": "10"}}],
            "networkInterfaces": [{"network": self.config.get("vpc", "global/networks/default"),
                                   "accessConfigs": [{"type": "ONE_TO_ONE_NAT", "name": "External NAT"}]}],
            "metadata": {"items": [{"key": "user-data", "value": gateway_cloud_init(configuration)},
                                   {"key": "ssh-keys", "value": f"ubuntu:{configuration.ssh_key_pub.strip()}"}]},
            "labels": merged_tags("gcp", {"owner": "dstack", "dstack_project": gcp_label(configuration.project_name),
                                          "role": "gateway"}, self.config),
        }
        r = check_response(self.http.post(f"{self.API}/projects/{self.project}/zones/{zone}/instances",
                                          headers=self._h(), json=body), "gcp gateway insert")
        self._wait_op(r, "gcp gateway insert")
        for _ in range(60):
            info = self._describe(name, configuration.region, {"zone": zone})
            if info.get("hostname"):
                return GatewayProvisioningData(instance_id=name, ip_address=info["hostname"],
                                               region=configuration.region, availability_zone=zone,
                                               backend_data=json.dumps({"zone": zone}))
            time.sleep(5)
        raise ComputeError(f"gcp gateway {name} got no external IP")

    def terminate_gateway(self, instance_id, configuration, backend_data=None):
        self._terminate(instance_id, configuration.region, json.loads(backend_data or "{}"))

    # ---- volumes: zonal persistent disks (reference ``C/backends/gcp/compute.py`` volumes) -------
    def _disk_url(self, zone: str, name: str = "") -> str:
        return f"{self.API}/projects/{self.project}/zones/{zone}/disks" + (f"/{name}" if name else "")

    @staticmethod
    def _volume_zone(volume) -> str:
        pd = volume.provisioning_data
        return (pd.availability_zone if pd and pd.availability_zone else None) or f"{volume.configuration.region}-a"

    def register_volume(self, volume):
        from dstack_amd.core.models.volumes import VolumeProvisioningData

        zone = self._zone(volume.configuration.region)
        r = self.http.get(self._disk_url(zone, volume.configuration.volume_id), headers=self._h())
        if r.status_code == 404:
            raise ComputeError(f"disk {volume.configuration.volume_id} not found in {zone}")
        d = check_response(r, "gcp get disk").json()
        return VolumeProvisioningData(backend=self.TYPE, volume_id=d["name"], size_gb=int(d.get("sizeGb", 0)),
                                      availability_zone=zone)

    def create_volume(self, volume):
        from dstack_amd.core.models.volumes import VolumeProvisioningData

        zone = self._zone(volume.configuration.region)
        size = int(volume.configuration.size or 100)
        name = f"{volume.name}-{str(volume.id)[:8]}".lower().replace("_", "-")[:62]
        body = {"name": name, "sizeGb": str(size), "type": f"zones/{zone}/diskTypes/"
                f"{self.config.get('volume_disk_type', 'pd-balanced')}",
                "labels": merged_tags("gcp", {"owner": "dstack", "dstack_project": gcp_label(volume.project_name)},
                                      self.config)}
        r = check_response(self.http.post(self._disk_url(zone), headers=self._h(), json=body), "gcp create disk")
        self._wait_op(r, "gcp create disk")
        return VolumeProvisioningData(backend=self.TYPE, volume_id=name, size_gb=size, availability_zone=zone,
                                      price=0.10 * size / 730)

    def delete_volume(self, volume):
        r = self.http.delete(self._disk_url(self._volume_zone(volume), volume.volume_id), headers=self._h())
        if r.status_code != 404:
            self._wait_op(check_response(r, "gcp delete disk"), "gcp delete disk")

    def attach_volume(self, volume, instance_id):
        from dstack_amd.core.models.volumes import VolumeAttachmentData

        zone = self._volume_zone(volume)
        body = {"source": f"projects/{self.project}/zones/{zone}/disks/{volume.volume_id}",
                "deviceName": volume.volume_id, "mode": "READ_WRITE", "autoDelete": False}
        r = check_response(self.http.post(f"{self.API}/projects/{self.project}/zones/{zone}/instances/"
                                          f"{instance_id}/attachDisk", headers=self._h(), json=body), "gcp attach")
        self._wait_op(r, "gcp attach disk")
        # the shim resolves /dev/disk/by-id/google-<device name> (native/shim/volumes.cpp)
        return VolumeAttachmentData(device_name=volume.volume_id)

    def detach_volume(self, volume, instance_id, force=False):
        zone = self._volume_zone(volume)
        r = self.http.post(f"{self.API}/projects/{self.project}/zones/{zone}/instances/{instance_id}/detachDisk"
                           f"?deviceName={urllib.parse.quote(volume.volume_id)}", headers=self._h())
        if r.status_code != 404:
            self._wait_op(check_response(r, "gcp detach"), "gcp detach disk")

    def is_volume_detached(self, volume, instance_id):
        r = self.http.get(self._disk_url(self._volume_zone(volume), volume.volume_id), headers=self._h())
        if r.status_code == 404:
            return True
        users = check_response(r, "gcp get disk").json().get("users") or []
        return not any(u.rstrip("/").endswith(f"/instances/{instance_id}") for u in users)


class ShapesQuota:
    """Which shapes the compartment may launch where: region -> availability domain -> shape
    names, as ``ListShapes`` reports per AD (reference ``C/backends/oci/resources.py:72-93``)."""

    def __init__(self, region_ads: Dict[str, Dict[str, set]]):
        self._by_ad = {ad: set(shapes) for ads in region_ads.values() for ad, shapes in ads.items()}
        self._by_region = {region: set().union(*ads.values()) if ads else set() for region, ads in region_ads.items()}
        self._ads = {region: sorted(ads) for region, ads in region_ads.items()}

    def is_within_region_quota(self, shape: str, region: str) -> bool:
        return shape in self._by_region.get(region, ())

    def is_within_domain_quota(self, shape: str, ad: str) -> bool:
        return shape in self._by_ad.get(ad, ())

    def domains_for(self, shape: str, region: str) -> List[str]:
        return [ad for ad in self._ads.get(region, []) if shape in self._by_ad[ad]]


@dataclass(frozen=True)
class SecurityRule:
    """A security-list rule reduced to what decides its effect, so rules read back from the API
    (with ids, timestamps, ``isStateless: false`` defaults, options objects) compare equal to the ones
    dstack wants (reference ``C/backends/oci/resources.py`` ``SecurityRule.from_sdk_rule``)."""

    direction: str  # "INGRESS" | "EGRESS"
    protocol: str  # "all", "6" (TCP), "17" (UDP), "1" (ICMP)
    peer: str  # source (ingress) / destination (egress) CIDR
    peer_type: str = "CIDR_BLOCK"
    is_stateless: bool = False
    ports: Optional[Tuple[int, int]] = None
    icmp: Optional[Tuple[int, Optional[int]]] = None

    @classmethod
    def from_api(cls, rule: dict, direction: str) -> "SecurityRule":
        ingress = direction == "INGRESS"
        opts = rule.get("tcpOptions") or rule.get("udpOptions") or {}
        rng = opts.get("destinationPortRange")
        icmp = rule.get("icmpOptions")
        return cls(direction=direction, protocol=str(rule.get("protocol", "all")),
                   peer=rule.get("source" if ingress else "destination", ""),
                   peer_type=rule.get("sourceType" if ingress else "destinationType") or "CIDR_BLOCK",
                   is_stateless=bool(rule.get("isStateless", False)),
                   ports=(int(rng["min"]), int(rng["max"])) if rng else None,
                   icmp=(int(icmp["type"]), icmp.get("code")) if icmp else None)

    def to_api(self) -> dict:
        ingress = self.direction == "INGRESS"
        d = {"protocol": self.protocol, ("source" if ingress else "destination"): self.peer,
             ("sourceType" if ingress else "destinationType"): self.peer_type, "isStateless": self.is_stateless}
        if self.ports:
            d["udpOptions" if self.protocol == "17" else "tcpOptions"] = {
                "destinationPortRange": {"min": self.ports[0], "max": self.ports[1]}}
        if self.icmp:
            d["icmpOptions"] = {"type": self.icmp[0], **({"code": self.icmp[1]} if self.icmp[1] is not None else {})}
        return d


# ---------------------------------------------------------------------------------------------
class OCICompute(VMCompute):
    TYPE = BackendType.OCI
    SSH_USER = "ubuntu"
    API_VERSION = "20160918"
    CONFIGURABLE_DISK = (50.0, 32768.0)  # boot volume, GB

    def _host(self, region: str) -> str:
        return f"iaas.{region}.oraclecloud.com"

    def _compartment(self) -> str:
        return self.config.get("compartment_id") or self.auth.get("tenancy")

    def check_credentials(self) -> None:
        # the identity API is asked in the key's home region (always subscribed)
        region = self.auth.get("region") or (self.config.get("regions") or ["us-ashburn-1"])[0]
        user = urllib.parse.quote(self.auth.get("user", ""))
        r = self._signed("GET", region, f"/{self.API_VERSION}/users/{user}", host=f"identity.{region}.oraclecloud.com")
        if r.status_code in (401, 403, 404):
            raise BackendAuthError(f"oci user: {r.status_code} {r.text[:200]}")
        check_response(r, "oci user")
        # every configured region must be subscribed by the tenancy (else launches fail later)
        wanted = self.config.get("regions") or []
        if wanted:
            tenancy = urllib.parse.quote(self.auth.get("tenancy", ""))
            r = check_response(self._signed("GET", region, f"/{self.API_VERSION}/tenancies/{tenancy}/regionSubscriptions",
                                            host=f"identity.{region}.oraclecloud.com"), "oci region subscriptions")
            subscribed = {x.get("regionName") for x in r.json()}
            missing = [x for x in wanted if x not in subscribed]
            if missing:
                raise ServerClientError(f"Regions {missing} are not subscribed by the OCI tenancy "
                                        f"(subscribed: {sorted(x for x in subscribed if x)})")

    # -- network bootstrap (reference ``oci/resources.py:427-690``) -------------------------------
    # One compartment for everything dstack creates (unless the config names one), and per region a
    # VCN with an internet gateway, a default route to it, security rules (SSH from anywhere, all
    # traffic inside the VCN -- RCCL/torch.distributed between nodes use ephemeral ports) and one
    # regional subnet.  Every step is get-or-create by display name, so it is idempotent and safe to
    # repeat at launch for regions added later.
    NET_NAME = "dstack"
    VCN_CIDR = "10.0.0.0/16"
    SUBNET_CIDR = "10.0.0.0/18"
    WAIT_S = 120.0
    WAIT_POLL_S = 2.0

    def _home_region(self) -> str:
        return self.auth.get("region") or (self.config.get("regions") or ["us-ashburn-1"])[0]

    def _identity(self, method: str, path: str, body: Optional[dict] = None):
        region = self._home_region()
        return self._signed(method, region, f"/{self.API_VERSION}{path}", body,
                            host=f"identity.{region}.oraclecloud.com")

    def _list_named(self, region: str, kind: str, name: str, **params) -> Optional[dict]:
        q = urllib.parse.urlencode({**params, "displayName": name})
        items = check_response(self._signed("GET", region, f"/{self.API_VERSION}/{kind}?{q}"), f"oci list {kind}").json()
        live = [x for x in items if x.get("lifecycleState") not in ("TERMINATED", "TERMINATING")]
        return live[0] if live else None

    def _wait_available(self, region: str, kind: str, obj: dict, host: Optional[str] = None) -> dict:
        deadline = time.time() + self.WAIT_S
        while obj.get("lifecycleState") not in ("AVAILABLE", "ACTIVE"):
            if time.time() > deadline:
                raise ComputeError(f"oci {kind} {obj.get('id')} still {obj.get('lifecycleState')}")
            time.sleep(self.WAIT_POLL_S)
            obj = check_response(self._signed("GET", region, f"/{self.API_VERSION}/{kind}/{obj['id']}", host=host),
                                 f"oci get {kind}").json()
        return obj

    def ensure_compartment(self) -> str:
        if self.config.get("compartment_id"):
            return self.config["compartment_id"]
        tenancy = self.auth["tenancy"]
        q = urllib.parse.urlencode({"compartmentId": tenancy, "name": self.NET_NAME, "lifecycleState": "ACTIVE"})
        found = check_response(self._identity("GET", f"/compartments?{q}"), "oci compartments").json()
        if found:
            comp = found[0]
        else:
            comp = check_response(self._identity("POST", "/compartments", {
                "compartmentId": tenancy, "name": self.NET_NAME,
                "description": "Resources created by dstack"}), "oci create compartment").json()
            region = self._home_region()
            comp = self._wait_available(region, "compartments", comp, host=f"identity.{region}.oraclecloud.com")
        self.config["compartment_id"] = comp["id"]
        return comp["id"]

    def ensure_network(self, region: str) -> str:
        """The subnet instances of ``region`` launch into (created on first use)."""
        comp = self.ensure_compartment()
        vcn = self._list_named(region, "vcns", f"{self.NET_NAME}-vcn", compartmentId=comp)
        if vcn is None:
            vcn = check_response(self._signed("POST", region, f"/{self.API_VERSION}/vcns", {
                "compartmentId": comp, "cidrBlocks": [self.VCN_CIDR], "displayName": f"{self.NET_NAME}-vcn",
                "dnsLabel": self.NET_NAME}), "oci create vcn").json()
        vcn = self._wait_available(region, "vcns", vcn)
        igw = self._list_named(region, "internetGateways", f"{self.NET_NAME}-igw", compartmentId=comp, vcnId=vcn["id"])
        if igw is None:
            igw = check_response(self._signed("POST", region, f"/{self.API_VERSION}/internetGateways", {
                "compartmentId": comp, "vcnId": vcn["id"], "isEnabled": True,
                "displayName": f"{self.NET_NAME}-igw"}), "oci create internet gateway").json()
        igw = self._wait_available(region, "internetGateways", igw)
        rt_id = vcn["defaultRouteTableId"]
        rt = check_response(self._signed("GET", region, f"/{self.API_VERSION}/routeTables/{rt_id}"), "oci route table").json()
        rules = rt.get("routeRules") or []
        if not any(r.get("destination") == "0.0.0.0/0" for r in rules):
            check_response(self._signed("PUT", region, f"/{self.API_VERSION}/routeTables/{rt_id}", {"routeRules": rules + [
                {"destination": "0.0.0.0/0", "destinationType": "CIDR_BLOCK", "networkEntityId": igw["id"]}]}),
                "oci update route table")
        sl_id = vcn["defaultSecurityListId"]
        self._ensure_security_rules(region, sl_id)
        subnet = self._list_named(region, "subnets", f"{self.NET_NAME}-subnet", compartmentId=comp, vcnId=vcn["id"])
        if subnet is None:
            subnet = check_response(self._signed("POST", region, f"/{self.API_VERSION}/subnets", {
                "compartmentId": comp, "vcnId": vcn["id"], "cidrBlock": self.SUBNET_CIDR,
                "displayName": f"{self.NET_NAME}-subnet", "dnsLabel": "nodes", "routeTableId": rt_id,
                "securityListIds": [sl_id], "prohibitPublicIpOnVnic": False}), "oci create subnet").json()
        subnet = self._wait_available(region, "subnets", subnet)
        self.config.setdefault("subnet_ids", {})[region] = subnet["id"]
        return subnet["id"]

    def required_security_rules(self) -> List[SecurityRule]:
        """SSH from anywhere, everything inside the VCN (RCCL/RDMA between nodes), path-MTU ICMP, any egress."""
        return [SecurityRule("INGRESS", "6", "0.0.0.0/0", ports=(22, 22)),
                SecurityRule("INGRESS", "all", self.VCN_CIDR),
                SecurityRule("INGRESS", "1", "0.0.0.0/0", icmp=(3, 4)),
                SecurityRule("EGRESS", "all", "0.0.0.0/0")]

    def _ensure_security_rules(self, region: str, sl_id: str) -> bool:
        """Add the rules dstack needs to the security list, keeping the ones already there;
        no update when all are present. True when the list was changed."""
        path = f"/{self.API_VERSION}/securityLists/{sl_id}"
        cur = check_response(self._signed("GET", region, path), "oci security list").json()
        have = {"INGRESS": [SecurityRule.from_api(r, "INGRESS") for r in cur.get("ingressSecurityRules") or []],
                "EGRESS": [SecurityRule.from_api(r, "EGRESS") for r in cur.get("egressSecurityRules") or []]}
        missing = [r for r in self.required_security_rules() if r not in have[r.direction]]
        if not missing:
            return False
        for r in missing:
            have[r.direction].append(r)
        check_response(self._signed("PUT", region, path, {
            "ingressSecurityRules": [r.to_api() for r in have["INGRESS"]],
            "egressSecurityRules": [r.to_api() for r in have["EGRESS"]]}), "oci update security list")
        return True

    def prepare_config(self) -> dict:
        """At backend creation: compartment + per-region networks, recorded in the stored config
        so launches go straight to them (regions without a configured subnet only)."""
        for region in self.config.get("regions") or [self._home_region()]:
            if not (self.config.get("subnet_ids") or {}).get(region):
                self.ensure_network(region)
        return {"compartment_id": self.config["compartment_id"], "subnet_ids": dict(self.config["subnet_ids"])}

    def _availability_domains(self, region: str) -> List[str]:
        """The tenancy's availability-domain names in ``region`` (tenancy-prefixed, e.g.
        ``Uocm:US-CHICAGO-1-AD-1``: they cannot be derived from the region name)."""
        q = urllib.parse.urlencode({"compartmentId": self.auth.get("tenancy") or self._compartment()})
        r = check_response(self._signed("GET", region, f"/{self.API_VERSION}/availabilityDomains?{q}",
                                        host=f"identity.{region}.oraclecloud.com"), "oci availability domains")
        return sorted(d["name"] for d in r.json())

    def _shapes(self, region: str, ad: str) -> List[str]:
        out, page = [], None
        for _ in range(50):
            params = {"compartmentId": self._compartment(), "availabilityDomain": ad, "limit": 100}
            if page:
                params["page"] = page
            r = check_response(self._signed("GET", region, f"/{self.API_VERSION}/shapes?"
                                            + urllib.parse.urlencode(params)), "oci shapes")
            out.extend(x.get("shape") for x in r.json())
            page = r.headers.get("opc-next-page")
            if not page:
                break
        return out

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Catalog shapes checked against the compartment's shapes per availability domain
        (``ListShapes``): shapes no AD of a region offers are ``not_available``; the ADs that offer
        each shape are remembered for the launch."""
        base = offline_rows(self.TYPE)
        wanted = self.config.get("regions")
        regions = sorted(set(wanted or []) | {r.location for r in base if not wanted})
        quota = ShapesQuota({region: {ad: set(self._shapes(region, ad)) for ad in self._availability_domains(region)}
                             for region in regions})
        self._quota = quota
        specs: Dict[Tuple[str, bool], CatalogRow] = {}
        for r in base:
            specs.setdefault((r.instance_name, r.spot), r)
        out = []
        for (name, spot), proto in sorted(specs.items()):
            for region in regions:
                out.append(replace(proto, location=region, availability=InstanceAvailability.UNKNOWN
                                   if quota.is_within_region_quota(name, region)
                                   else InstanceAvailability.NOT_AVAILABLE))
        return out

    def _ad_for(self, region: str, shape: str) -> str:
        ads = self.config.get("availability_domains") or {}
        if ads.get(region):
            return ads[region]
        quota = getattr(self, "_quota", None)
        offered = quota.domains_for(shape, region) if quota else []
        if offered:
            return offered[0]
        for ad in self._availability_domains(region):
            if shape in self._shapes(region, ad):
                return ad
        raise ComputeError(f"no availability domain of {region} offers {shape}")

    def _signed(self, method: str, region: str, path: str, body: Optional[dict] = None, host: Optional[str] = None):
        host = host or self._host(region)
        date = email.utils.formatdate(usegmt=True)
        headers = {"date": date, "host": host}
        data = b""
        names = ["(request-target)", "date", "host"]
        if body is not None:
            data = json.dumps(body).encode()
            headers.update({"content-type": "application/json", "content-length": str(len(data)),
                            "x-content-sha256": base64.b64encode(hashlib.sha256(data).digest()).decode()})
            names += ["x-content-sha256", "content-type", "content-length"]
        lines = []
        for n in names:
            lines.append(f"(request-target): {method.lower()} {path}" if n == "(request-target)" else f"{n}: {headers[n]}")
        sig = base64.b64encode(rsa_sha256_sign(self.auth["key_content"], "\n".join(lines).encode())).decode()
        key_id = f"{self.auth['tenancy']}/{self.auth['user']}/{self.auth['fingerprint']}"
        headers["authorization"] = (f'Signature version="1",keyId="{key_id}",algorithm="rsa-sha256",'
                                    f'headers="{" ".join(names)}",signature="{sig}"')
        return self.http.request(method, f"https://{host}{path}", headers=headers, content=data or None)

    def _launch(self, offer, cfg):
        region = offer.region
        subnet = (self.config.get("subnet_ids") or {}).get(region) or self.ensure_network(region)
        comp = self._compartment()
        body = {
            "compartmentId": comp, "availabilityDomain": self._ad_for(region, offer.instance.name),
            "shape": offer.instance.name,
            "displayName": cfg.instance_name,
            "sourceDetails": {"sourceType": "image", "imageId": self._image_id(region, comp, offer.instance.name),
                              "bootVolumeSizeInGBs": max(100, offer.instance.resources.disk.size_mib // 1024)},
            "createVnicDetails": {"subnetId": subnet, "assignPublicIp": True},
            "metadata": {"ssh_authorized_keys": "\n".join(cfg.get_public_keys()),
                         "user_data": base64.b64encode(cloud_init(cfg).encode()).decode()},
        }
        if offer.instance.resources.spot:
            body["preemptibleInstanceConfig"] = {"preemptionAction": {"type": "TERMINATE", "preserveBootVolume": False}}
        r = check_response(self._signed("POST", region, f"/{self.API_VERSION}/instances", body), "oci launch")
        return r.json()["id"], None, {"compartment": comp}

    def _image_id(self, region: str, compartment: str, shape: str) -> str:
        """The configured image, else the newest Canonical Ubuntu 22.04 image compatible with the
        shape (the GPU bare-metal shapes need their own image builds, so the shape filter matters)."""
        img = (self.config.get("images") or {}).get(region)
        if img:
            return img
        q = urllib.parse.urlencode({"compartmentId": compartment, "operatingSystem": "Canonical Ubuntu",
                                    "operatingSystemVersion": "22.04", "shape": shape, "sortBy": "TIMECREATED",
                                    "sortOrder": "DESC", "lifecycleState": "AVAILABLE"})
        items = check_response(self._signed("GET", region, f"/{self.API_VERSION}/images?{q}"), "oci images").json()
        if not items:
            raise ComputeError(f"no Ubuntu 22.04 image for shape {shape} in {region}; set images.{region}")
        return items[0]["id"]

    def _describe(self, instance_id, region, backend_data):
        r = self._signed("GET", region, f"/{self.API_VERSION}/instances/{urllib.parse.quote(instance_id)}")
        if r.status_code == 404:
            return {"status": "terminated"}
        st = check_response(r, "oci get").json().get("lifecycleState", "").lower()
        if st != "running":
            return {"status": st}
        q = urllib.parse.urlencode({"compartmentId": backend_data.get("compartment", ""), "instanceId": instance_id})
        att = check_response(self._signed("GET", region, f"/{self.API_VERSION}/vnicAttachments?{q}"), "oci vnics").json()
        if not att:
            return {"status": st}
        vnic = check_response(self._signed("GET", region, f"/{self.API_VERSION}/vnics/{att[0]['vnicId']}"),
                              "oci vnic").json()
        return {"status": st, "hostname": vnic.get("publicIp"), "internal_ip": vnic.get("privateIp")}

    def _terminate(self, instance_id, region, backend_data):
        r = self._signed("DELETE", region, f"/{self.API_VERSION}/instances/{urllib.parse.quote(instance_id)}")
        if r.status_code not in (200, 204, 404):
            check_response(r, "oci terminate")

