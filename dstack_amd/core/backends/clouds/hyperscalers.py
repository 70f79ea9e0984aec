"""Azure, GCP and OCI over their REST APIs (reference: ``C/backends/azure/compute.py`` (839 LoC,
azure-mgmt SDK), ``C/backends/gcp/compute.py`` (1378, google-cloud SDK), ``C/backends/oci/compute.py``
(1181, oci SDK)).

* Azure: OAuth2 client credentials -> one ARM template deployment per VM (public IP + NIC + VM with
  cloud-init ``customData``); the MI300X path is ``Standard_ND96isr_MI300X_v5``.
* GCP: service-account JWT (RS256 via OpenSSL) -> ``instances.insert`` with a NAT access config.
* OCI: HTTP-signature auth (RSA-SHA256 via OpenSSL) -> ``LaunchInstance``; the ``BM.GPU.MI300X.8``
  bare-metal shape takes up to 20 minutes to boot (the reference's 1200 s timeout).
"""

from __future__ import annotations

import base64
import email.utils
import hashlib
import json
import time
import urllib.parse
from typing import Dict, Optional, Tuple

from dstack_amd.core.backends.clouds.common import (
    OAuthToken,
    VMCompute,
    b64url,
    check_response,
    cloud_init,
    rsa_sha256_sign,
)
from dstack_amd.core.errors import ComputeError
from dstack_amd.core.models.backends import BackendType


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
        r = check_response(self.http.post(
            f"https://login.microsoftonline.com/{self.tenant}/oauth2/v2.0/token",
            data={"grant_type": "client_credentials", "client_id": self.auth.get("client_id"),
                  "client_secret": self.auth.get("client_secret"), "scope": f"{self.ARM}/.default"}), "azure token")
        d = r.json()
        return d["access_token"], d.get("expires_in", 3600)

    def _h(self):
        return {"Authorization": f"Bearer {self._token.get()}"}

    def _rg(self, region: str) -> str:
        rg = (self.config.get("resource_groups") or {}).get(region) or f"dstack-{region}"
        url = f"{self.ARM}/subscriptions/{self.subscription}/resourcegroups/{rg}?api-version=2021-04-01"
        check_response(self.http.put(url, headers=self._h(), json={"location": region}), "azure resource group")
        return rg

    def _template(self, name: str, size: str, region: str, user_data: str, disk_gb: int, spot: bool,
                  public_keys) -> dict:
        subnet = self.config.get("subnet_id") or (
            f"[resourceId('Microsoft.Network/virtualNetworks/subnets', 'dstack-vnet-{region}', 'default')]")
        vm_props = {
            "hardwareProfile": {"vmSize": size},
            "storageProfile": {"imageReference": {"publisher": "Canonical", "offer": "0001-com-ubuntu-server-jammy",
                                                  "sku": "22_04-lts-gen2", "version": "latest"},
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
        res = [
            {"type": "Microsoft.Network/publicIPAddresses", "apiVersion": "2023-04-01", "name": f"{name}-ip",
             "location": region, "sku": {"name": "Standard"}, "properties": {"publicIPAllocationMethod": "Static"}},
            {"type": "Microsoft.Network/networkInterfaces", "apiVersion": "2023-04-01", "name": f"{name}-nic",
             "location": region, "dependsOn": [f"[resourceId('Microsoft.Network/publicIPAddresses', '{name}-ip')]"],
             "properties": {"enableAcceleratedNetworking": True, "ipConfigurations": [{"name": "ipconfig1", "properties": {
                 "subnet": {"id": subnet}, "publicIPAddress": {"id": f"[resourceId('Microsoft.Network/"
                                                                       f"publicIPAddresses', '{name}-ip')]"}}}]}},
            {"type": "Microsoft.Compute/virtualMachines", "apiVersion": "2023-03-01", "name": name, "location": region,
             "dependsOn": [f"[resourceId('Microsoft.Network/networkInterfaces', '{name}-nic')]"],
             "properties": vm_props},
        ]
        return {"$schema": "https://schema.management.azure.com/schemas/2019-04-01/deploymentTemplate.json#",
                "contentVersion": "1.0.0.0", "resources": res}

    def _launch(self, offer, cfg):
        region = offer.region
        rg = self._rg(region)
        name = cfg.instance_name.replace("_", "-")[:60]
        tpl = self._template(name, offer.instance.name, region, cloud_init(cfg),
                             max(100, offer.instance.resources.disk.size_mib // 1024), offer.instance.resources.spot,
                             cfg.get_public_keys())
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
        for path, ver in ((f"Microsoft.Compute/virtualMachines/{instance_id}", "2023-03-01"),
                          (f"Microsoft.Network/publicIPAddresses/{instance_id}-ip", "2023-04-01")):
            r = self.http.delete(f"{base}/{path}?api-version={ver}", headers=self._h())
            if r.status_code not in (200, 202, 204, 404):
                check_response(r, f"azure delete {path}")


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
        r = check_response(self.http.post("https://oauth2.googleapis.com/token", data={
            "grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer", "assertion": f"{header}.{claims}.{sig}"}),
            "gcp token")
        d = r.json()
        return d["access_token"], d.get("expires_in", 3600)

    def _h(self):
        return {"Authorization": f"Bearer {self._token.get()}"}

    def _zone(self, region: str) -> str:
        zones = self.config.get("zones") or {}
        return zones.get(region) or f"{region}-a"

    def _launch(self, offer, cfg):
        zone = self._zone(offer.region)
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
            "labels": {"owner": "dstack", "dstack_project": cfg.project_name.lower()},
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


# ---------------------------------------------------------------------------------------------
class OCICompute(VMCompute):
    TYPE = BackendType.OCI
    SSH_USER = "ubuntu"
    API_VERSION = "20160918"

    def _host(self, region: str) -> str:
        return f"iaas.{region}.oraclecloud.com"

    def _signed(self, method: str, region: str, path: str, body: Optional[dict] = None):
        host = self._host(region)
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
        comp = self.config.get("compartment_id") or self.auth.get("tenancy")
        ads = self.config.get("availability_domains") or {}
        body = {
            "compartmentId": comp, "availabilityDomain": ads.get(region, f"{region}-AD-1"), "shape": offer.instance.name,
            "displayName": cfg.instance_name,
            "sourceDetails": {"sourceType": "image", "imageId": (self.config.get("images") or {}).get(region, ""),
                              "bootVolumeSizeInGBs": max(100, offer.instance.resources.disk.size_mib // 1024)},
            "createVnicDetails": {"subnetId": (self.config.get("subnet_ids") or {}).get(region), "assignPublicIp": True},
            "metadata": {"ssh_authorized_keys": "\n".join(cfg.get_public_keys()),
                         "user_data": base64.b64encode(cloud_init(cfg).encode()).decode()},
        }
        if offer.instance.resources.spot:
            body["preemptibleInstanceConfig"] = {"preemptionAction": {"type": "TERMINATE", "preserveBootVolume": False}}
        r = check_response(self._signed("POST", region, f"/{self.API_VERSION}/instances", body), "oci launch")
        return r.json()["id"], None, {"compartment": comp}

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


_ = (Dict, Tuple, ComputeError)
