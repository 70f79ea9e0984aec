"""REST-API VM clouds (reference: ``C/backends/{lambdalabs,vultr,tensordock,cudo,datacrunch,nebius}/
compute.py`` and their ``api_client.py``).

Each class maps the cloud's launch / get / terminate endpoints onto ``VMCompute``; the VM's
cloud-init installs ``dstack-shim``.  Vultr is the MI355X/MI325X/MI300X bare-metal path.
"""

from __future__ import annotations

import base64
import re
import uuid
from typing import Dict, List, Optional, Tuple

from dstack_amd.core.backends.catalog import CatalogRow, gpu_row
from dstack_amd.core.backends.clouds.common import (
    OAuthToken,
    VMCompute,
    check_response,
    cloud_init,
    ssh_key_fingerprint,
)
from dstack_amd.core.errors import BackendAuthError, ComputeError, NoCapacityError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gpus import gpu_info, normalize_gpu_name
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceConfiguration,
    InstanceOfferWithAvailability,
)

_AVAILABLE, _NOT_AVAILABLE = InstanceAvailability.AVAILABLE, InstanceAvailability.NOT_AVAILABLE


class LambdaCompute(VMCompute):
    """Lambda Cloud: ``/instance-operations/launch`` + registered SSH key (lambdalabs/compute.py)."""

    TYPE = BackendType.LAMBDA
    API = "https://cloud.lambdalabs.com/api/v1"

    REGIONS = ("us-east-1", "us-east-2", "us-west-1", "us-west-2", "us-west-3", "us-south-1", "us-south-2",
               "us-south-3", "us-midwest-1", "europe-central-1", "asia-northeast-1", "asia-northeast-2",
               "asia-south-1", "me-west-1")

    def _h(self):
        return {"Authorization": f"Bearer {self.auth.get('api_key', '')}"}

    def _fetch_catalog(self) -> List[CatalogRow]:
        """``GET /instance-types``: price, specs and the regions with capacity right now.  Regions
        without capacity are listed as ``not_available`` so the plan still shows the type."""
        r = check_response(self.http.get(f"{self.API}/instance-types", headers=self._h()), "lambda instance-types")
        rows = []
        for key, d in (r.json().get("data") or {}).items():
            it = d.get("instance_type") or {}
            specs = it.get("specs") or {}
            m = re.match(r"\s*([A-Za-z0-9]+)[^(]*(?:\((\d+)\s*GB)?", it.get("gpu_description") or "")
            gpu_name = m.group(1) if m and specs.get("gpus") else None
            gpu_mem = float(m.group(2)) if m and m.group(2) else None
            with_capacity = {x.get("name") for x in d.get("regions_with_capacity_available") or []}
            for loc in sorted(with_capacity | set(self.config.get("regions") or self.REGIONS)):
                rows.append(gpu_row(it.get("name", key), loc, float(it.get("price_cents_per_hour", 0)) / 100,
                                    specs.get("vcpus", 0), specs.get("memory_gib", 0), gpu_name,
                                    specs.get("gpus", 0), disk_gb=specs.get("storage_gib"), gpu_memory_gb=gpu_mem,
                                    availability=_AVAILABLE if loc in with_capacity else _NOT_AVAILABLE))
        return rows

    def check_credentials(self) -> None:
        check_response(self.http.get(f"{self.API}/instance-types", headers=self._h()), "lambda instance-types")

    def _ensure_keys(self, cfg: InstanceConfiguration) -> List[str]:
        """Account SSH keys for the instance's public keys: an account key with the same fingerprint
        is reused whatever its name, otherwise the key is added as ``dstack-<fingerprint tail>`` (a
        name per key, so two projects never fight over one name; lambdalabs/compute.py
        ``_add_project_ssh_key`` names keys by a hash of the key as well)."""
        r = check_response(self.http.get(f"{self.API}/ssh-keys", headers=self._h()), "lambda ssh-keys")
        have = {}
        for k in r.json().get("data", []):
            try:
                have[ssh_key_fingerprint(k.get("public_key", ""))] = k["name"]
            except (ValueError, IndexError):
                continue
        names = []
        for pk in cfg.get_public_keys():
            fp = ssh_key_fingerprint(pk)
            if fp not in have:
                name = "dstack-" + re.sub(r"[^A-Za-z0-9]", "", fp.split(":", 1)[1])[-16:]
                check_response(self.http.post(f"{self.API}/ssh-keys", headers=self._h(),
                                              json={"name": name, "public_key": pk.strip()}), "lambda add ssh-key")
                have[fp] = name
            names.append(have[fp])
        return list(dict.fromkeys(names))

    def _launch(self, offer: InstanceOfferWithAvailability, cfg: InstanceConfiguration
                ) -> Tuple[str, Optional[str], Optional[dict]]:
        body = {"region_name": offer.region, "instance_type_name": offer.instance.name,
                "ssh_key_names": self._ensure_keys(cfg), "name": cfg.instance_name, "quantity": 1,
                "user_data": cloud_init(cfg)}
        r = self.http.post(f"{self.API}/instance-operations/launch", headers=self._h(), json=body)
        if r.status_code == 400 and "insufficient-capacity" in r.text:
            raise NoCapacityError(f"lambda: no {offer.instance.name} capacity in {offer.region}")
        check_response(r, "lambda launch")
        return r.json()["data"]["instance_ids"][0], None, None

    def _describe(self, instance_id, region, backend_data) -> dict:
        r = self.http.get(f"{self.API}/instances/{instance_id}", headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        d = check_response(r, "lambda get").json()["data"]
        return {"status": d.get("status"), "hostname": d.get("ip"), "internal_ip": d.get("private_ip")}

    def _terminate(self, instance_id, region, backend_data) -> None:
        check_response(self.http.post(f"{self.API}/instance-operations/terminate", headers=self._h(),
                                      json={"instance_ids": [instance_id]}), "lambda terminate")


class VultrCompute(VMCompute):
    """Vultr v2 API: cloud GPU instances and bare metal (the MI300X/MI325X/MI355X 8-GPU nodes)."""

    TYPE = BackendType.VULTR
    API = "https://api.vultr.com/v2"
    SSH_USER = "root"
    UBUNTU_22_OS_ID = 1743

    def _h(self):
        return {"Authorization": f"Bearer {self.auth.get('api_key', '')}"}

    @staticmethod
    def _kind(plan: str) -> str:
        return "bare-metals" if plan.startswith("vbm-") else "instances"

    def check_credentials(self) -> None:
        check_response(self.http.get(f"{self.API}/account", headers=self._h()), "vultr account")

    def _list(self, path: str, key: str) -> List[dict]:
        out, cursor = [], ""
        for _ in range(50):
            params = {"per_page": 500, **({"cursor": cursor} if cursor else {})}
            d = check_response(self.http.get(f"{self.API}/{path}", params=params, headers=self._h()),
                               f"vultr {path}").json()
            out.extend(d.get(key) or [])
            cursor = ((d.get("meta") or {}).get("links") or {}).get("next") or ""
            if not cursor:
                break
        return out

    @staticmethod
    def _plan_gpu(plan: dict) -> Tuple[Optional[str], int, Optional[float]]:
        """GPU model / count / per-GPU memory of a plan: cloud GPU plans carry ``gpu_type`` +
        ``gpu_vram_gb``; bare metal encodes it in the id (``vbm-256c-2048gb-8-mi355x-gpu``)."""
        if plan.get("gpu_type"):
            name = str(plan["gpu_type"]).replace("NVIDIA_", "").replace("AMD_", "").split("_")[0]
            count = int(plan.get("gpu_count") or 1)
            vram = float(plan.get("gpu_vram_gb") or 0) / count or None
            return name, count, vram
        m = re.search(r"-(\d+)-([a-z0-9]+)-gpu$", plan.get("id", ""))
        if m:
            return m.group(2).upper(), int(m.group(1)), None
        return None, 0, None

    def _fetch_catalog(self) -> List[CatalogRow]:
        """GPU plans (``/plans?type=vcg``) and bare-metal plans (``/plans-metal``) with their hourly
        price, and per-region stock from ``/regions/{id}/availability``."""
        plans = [(p, False) for p in self._list("plans", "plans") if p.get("type") == "vcg" or p.get("gpu_type")]
        plans += [(p, True) for p in self._list("plans-metal", "plans_metal")]
        wanted = set(self.config.get("regions") or [])
        rows, stock = [], {}
        for plan, metal in plans:
            gpu_name, count, vram = self._plan_gpu(plan)
            if not gpu_name and not metal:
                continue
            full = gpu_info(normalize_gpu_name(gpu_name)) if gpu_name else None
            if vram is not None and full is not None and vram < 0.9 * full.memory_gb:
                continue  # fractional (vGPU) slice of a card
            price = plan.get("hourly_cost") or round(float(plan.get("monthly_cost", 0)) / 730, 4)
            for loc in plan.get("locations") or []:
                if wanted and loc not in wanted:
                    continue
                if loc not in stock:
                    d = check_response(self.http.get(f"{self.API}/regions/{loc}/availability", params={"type": "all"},
                                                     headers=self._h()), "vultr availability").json()
                    stock[loc] = set(d.get("available_plans") or [])
                cpus = plan.get("cpu_threads") or plan.get("cpu_count") or plan.get("vcpu_count") or 0
                rows.append(gpu_row(plan["id"], loc, float(price), cpus, float(plan.get("ram", 0)) / 1024, gpu_name,
                                    count, disk_gb=float(plan.get("disk", 0)) * int(plan.get("disk_count") or 1),
                                    gpu_memory_gb=vram,
                                    availability=_AVAILABLE if plan["id"] in stock[loc] else _NOT_AVAILABLE))
        return rows

    def _ensure_vpc(self, region: str) -> dict:
        """The region's dstack VPC (get or create): every instance and bare-metal node launches
        into it, so the nodes of a cluster reach each other privately (RCCL bootstrap, torchrun
        rendezvous) -- the public interface only carries SSH."""
        name = f"dstack-vpc-{region}"
        for vpc in self._list("vpcs", "vpcs"):
            if vpc.get("description") == name and vpc.get("region") in (None, region):
                return vpc
        return check_response(self.http.post(f"{self.API}/vpcs", headers=self._h(),
                                             json={"region": region, "description": name}), "vultr create vpc").json()["vpc"]

    def _launch(self, offer, cfg):
        kind = self._kind(offer.instance.name)
        vpc = self._ensure_vpc(offer.region)
        subnet = f"{vpc.get('v4_subnet')}/{vpc.get('v4_subnet_mask')}" if vpc.get("v4_subnet") else None
        # Vultr images ship ufw enabled: let the VPC subnet in (no-op where ufw is absent)
        host_cmds = [f"command -v ufw >/dev/null && ufw allow from {subnet} && ufw reload || true"] if subnet else []
        image = self.config.get("images") or {}
        body = {"region": offer.region, "plan": offer.instance.name, "label": cfg.instance_name,
                "user_data": base64.b64encode(cloud_init(cfg, host_cmds).encode()).decode(),
                "tags": ["dstack", cfg.project_name], "attach_vpc": [vpc["id"]]}
        # the OS: Ubuntu 22.04 unless ``images.{instance,bare_metal}`` names an OS id (digits) or a
        # marketplace image (e.g. a ROCm image for the AMD bare-metal plans)
        img = str(image.get("bare_metal" if kind == "bare-metals" else "instance") or self.UBUNTU_22_OS_ID)
        if img.isdigit():
            body["os_id"] = int(img)
        else:
            body["image_id"] = img
        if kind == "instances":
            body["backups"] = "disabled"
        r = check_response(self.http.post(f"{self.API}/{kind}", headers=self._h(), json=body), "vultr create")
        key = "bare_metal" if kind == "bare-metals" else "instance"
        return r.json()[key]["id"], None, {"kind": kind, "vpc_id": vpc["id"], "vpc_subnet": subnet}

    def _describe(self, instance_id, region, backend_data):
        kind = backend_data.get("kind", "instances")
        r = self.http.get(f"{self.API}/{kind}/{instance_id}", headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        d = check_response(r, "vultr get").json()
        d = d.get("bare_metal") or d.get("instance") or {}
        ip = d.get("main_ip")
        ready = d.get("status") == "active" and ip and ip != "0.0.0.0"
        internal = d.get("internal_ip") or None
        if ready and not internal and backend_data.get("vpc_id"):
            # the node's address in the dstack VPC is what its cluster peers connect to
            v = self.http.get(f"{self.API}/{kind}/{instance_id}/vpcs", headers=self._h())
            if v.status_code == 200:
                internal = next((x.get("ip_address") for x in v.json().get("vpcs") or []
                                 if x.get("id") == backend_data["vpc_id"]), None)
        return {"status": d.get("status"), "hostname": ip if ready else None, "internal_ip": internal}

    def _terminate(self, instance_id, region, backend_data):
        kind = backend_data.get("kind", "instances")
        r = self.http.delete(f"{self.API}/{kind}/{instance_id}", headers=self._h())
        if r.status_code != 404:
            check_response(r, "vultr delete")


class TensorDockCompute(VMCompute):
    """TensorDock marketplace: ``/client/deploy/single`` on a host node (tensordock/compute.py)."""

    TYPE = BackendType.TENSORDOCK
    API = "https://marketplace.tensordock.com/api/v0"
    SSH_USER = "user"

    CONFIGURABLE_DISK = (20.0, None)
    GPU_COUNTS = (1, 2, 4, 8)

    def _auth(self):
        return {"api_key": self.auth.get("api_key", ""), "api_token": self.auth.get("api_token", "")}

    def check_credentials(self) -> None:
        r = check_response(self.http.post(f"{self.API}/auth/test", data=self._auth()), "tensordock auth")
        if not (r.json() or {}).get("success"):
            raise BackendAuthError(f"tensordock: {r.text[:200]}")

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Marketplace host nodes (``/client/deploy/hostnodes``): one row per (GPU model, count)
        that fits a node, CPU / RAM in proportion to the GPUs taken, price = the node's per-unit
        GPU + vCPU + RAM + 100 GB disk prices.  Instance name ``<gpu model>:<count>:<node id>``."""
        r = check_response(self.http.get(f"{self.API}/client/deploy/hostnodes"), "tensordock hostnodes")
        rows = []
        for node_id, node in (r.json().get("hostnodes") or {}).items():
            if (node.get("status") or {}).get("online") is False:
                continue
            loc = node.get("location") or {}
            region = "-".join(str(x) for x in (loc.get("country"), loc.get("region"), loc.get("city")) if x)
            region = region.lower().replace(" ", "") or "any"
            specs = node.get("specs") or {}
            cpu, ram, disk = specs.get("cpu") or {}, specs.get("ram") or {}, specs.get("storage") or {}
            for model, g in (specs.get("gpu") or {}).items():
                avail = int(g.get("amount") or 0)
                for n in self.GPU_COUNTS:
                    if n > avail:
                        break
                    cpus = max(1, int(cpu.get("amount", 0)) * n // avail // 2 * 2)
                    mem = max(1, int(ram.get("amount", 0)) * n // avail)
                    if int(disk.get("amount", 0)) < 100:
                        continue
                    price = (n * float(g.get("price", 0)) + cpus * float(cpu.get("price", 0))
                             + mem * float(ram.get("price", 0)) + 100 * float(disk.get("price", 0)))
                    rows.append(gpu_row(f"{model}:{n}:{node_id}", region, price, cpus, mem,
                                        model.split("-")[0].upper(), n, gpu_memory_gb=g.get("vram"),
                                        availability=_AVAILABLE))
        return rows

    def _launch(self, offer, cfg):
        res = offer.instance.resources
        parts = offer.instance.name.split(":")
        node = parts[-1] if len(parts) > 1 else offer.region
        model = parts[0] if len(parts) == 3 else (res.gpus[0].name.lower() if res.gpus else "")
        data = {**self._auth(), "hostnode": node, "name": cfg.instance_name, "gpu_count": len(res.gpus),
                "gpu_model": model, "vcpus": res.cpus,
                "ram": res.memory_mib // 1024, "storage": res.disk.size_mib // 1024,
                "external_ports": "{22}", "internal_ports": "{22}", "operating_system": "Ubuntu 22.04 LTS",
                # the form field takes the cloud-config with its newlines escaped (tensordock/api_client.py)
                "cloudinit_script": cloud_init(cfg).replace("\n", "\\n"), "password": uuid.uuid4().hex}
        r = check_response(self.http.post(f"{self.API}/client/deploy/single", data=data), "tensordock deploy")
        d = r.json()
        if not d.get("success"):
            raise ComputeError(f"tensordock deploy: {d}")
        ssh_port = next((int(k) for k, v in (d.get("port_forwards") or {}).items() if str(v) == "22"), 22)
        return d["server"], d.get("ip"), {"ssh_port": ssh_port}

    def create_instance(self, instance_offer, instance_config):
        jpd = super().create_instance(instance_offer, instance_config)
        jpd.ssh_port = (eval_json(jpd.backend_data) or {}).get("ssh_port", 22)
        return jpd

    def _describe(self, instance_id, region, backend_data):
        r = check_response(self.http.post(f"{self.API}/client/get/single",
                                          data={**self._auth(), "server": instance_id}), "tensordock get")
        vm = r.json().get("virtualmachines") or {}
        return {"status": vm.get("status"), "hostname": vm.get("ip_address")}

    def _terminate(self, instance_id, region, backend_data):
        check_response(self.http.post(f"{self.API}/client/delete/single",
                                      data={**self._auth(), "server": instance_id}), "tensordock delete")


class CudoCompute(VMCompute):
    """Cudo Compute REST (cudo/compute.py): ``/projects/{p}/vm`` create/get/terminate."""

    TYPE = BackendType.CUDO
    API = "https://rest.compute.cudo.org/v1"
    SSH_USER = "root"

    def _h(self):
        return {"Authorization": f"Bearer {self.auth.get('api_key', '')}"}

    def check_credentials(self) -> None:
        check_response(self.http.get(f"{self.API}/projects/{self.config.get('project_id', 'default')}",
                                     headers=self._h()), "cudo project")

    def _image(self, res) -> str:
        """Boot image: ``images`` in the backend config by kind (``amd`` / ``nvidia`` / ``cpu``),
        else Cudo's NVIDIA driver + Docker image for NVIDIA GPUs and plain Ubuntu 22.04 otherwise
        (the AMD host setup installs the amdgpu/ROCm user space itself)."""
        vendor = getattr(res.gpus[0].vendor, "value", res.gpus[0].vendor) if res.gpus else None
        kind = "cpu" if not res.gpus else ("amd" if vendor == "amd" else "nvidia")
        over = (self.config.get("images") or {}).get(kind)
        if over:
            return over
        return "ubuntu-2204-nvidia-535-docker-v20240214" if kind == "nvidia" else "ubuntu-2204"

    # Cudo error codes on VM create (cudo/compute.py create_instance)
    NO_HOSTS, DISK_EXISTS, NETWORK_FULL = 3, 6, 9

    def _launch(self, offer, cfg):
        """``startScript`` is a plain shell script on Cudo (not cloud-config), so the bootstrap's
        runcmd lines are sent as one; the VM id carries the data centre so that the same instance
        name can be retried elsewhere; "no hosts available" is a capacity error, the rest fail."""
        project = self.config.get("project_id", "default")
        res = offer.instance.resources
        vm_id = f"{cfg.instance_name}-{offer.region}"[:60]
        script = "#!/bin/bash\n" + _runcmd_script(cloud_init(cfg))
        body = {"dataCenterId": offer.region, "machineType": offer.instance.name, "vmId": vm_id,
                "vcpus": res.cpus, "memoryGib": res.memory_mib // 1024, "gpus": len(res.gpus),
                "bootDiskImageId": self._image(res),
                "bootDisk": {"storageClass": "STORAGE_CLASS_NETWORK", "sizeGib": res.disk.size_mib // 1024,
                             "id": f"{vm_id}-disk"},
                "customSshKeys": cfg.get_public_keys(), "startScript": script}
        r = self.http.post(f"{self.API}/projects/{project}/vm", headers=self._h(), json=body)
        if r.status_code >= 400:
            try:
                d = r.json()
            except ValueError:
                d = {}
            if d.get("code") == self.NO_HOSTS:
                raise NoCapacityError(f"cudo: {d.get('message') or 'no hosts available'}")
            raise ComputeError(f"cudo create: HTTP {r.status_code} {d.get('message') or r.text[:200]}")
        return vm_id, None, {"project": project}

    def _describe(self, instance_id, region, backend_data):
        r = self.http.get(f"{self.API}/projects/{backend_data.get('project', 'default')}/vms/{instance_id}",
                          headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        vm = check_response(r, "cudo get").json().get("VM", {})
        return {"status": vm.get("state", "").lower(), "hostname": vm.get("externalIpAddress"),
                "internal_ip": vm.get("internalIpAddress")}

    def _terminate(self, instance_id, region, backend_data):
        r = self.http.post(f"{self.API}/projects/{backend_data.get('project', 'default')}/vms/{instance_id}/terminate",
                           headers=self._h())
        if r.status_code != 404:
            check_response(r, "cudo terminate")


class DataCrunchCompute(VMCompute):
    """DataCrunch: OAuth2 client credentials + ``/instances`` (datacrunch/compute.py)."""

    TYPE = BackendType.DATACRUNCH
    API = "https://api.datacrunch.io/v1"
    SSH_USER = "root"

    def __init__(self, config, auth, client=None):
        super().__init__(config, auth, client)
        self._token = OAuthToken(self._fetch_token)

    def _fetch_token(self):
        r = self.http.post(f"{self.API}/oauth2/token", json={
            "grant_type": "client_credentials", "client_id": self.auth.get("client_id"),
            "client_secret": self.auth.get("client_secret")})
        if r.status_code in (400, 401, 403):
            raise BackendAuthError(f"datacrunch token: {r.status_code} {r.text[:200]}")
        check_response(r, "datacrunch token")
        d = r.json()
        return d["access_token"], d.get("expires_in", 3600)

    def _h(self):
        return {"Authorization": f"Bearer {self._token.get()}"}

    CONFIGURABLE_DISK = (50.0, None)

    def check_credentials(self) -> None:
        self._token.get()  # the client-credentials exchange is the check

    def _fetch_catalog(self) -> List[CatalogRow]:
        """``/instance-types`` (on-demand and spot prices, specs) x ``/instance-availability`` per
        location, on-demand and spot separately."""
        types = check_response(self.http.get(f"{self.API}/instance-types", headers=self._h()),
                               "datacrunch instance-types").json()
        stock: Dict[Tuple[str, bool], set] = {}
        for spot in (False, True):
            av = check_response(self.http.get(f"{self.API}/instance-availability",
                                              params={"is_spot": str(spot).lower()}, headers=self._h()),
                                "datacrunch availability").json()
            for loc in av:
                stock[(loc.get("location_code"), spot)] = set(loc.get("availabilities") or [])
        locations = sorted({loc for loc, _ in stock} | set(self.config.get("regions") or []))
        rows = []
        for t in types:
            name = t.get("instance_type")
            gpu = t.get("gpu") or {}
            desc = re.sub(r"^\d+x\s*", "", gpu.get("description") or "")
            gpu_name = desc.split()[0] if desc and gpu.get("number_of_gpus") else None
            gpu_mem = (t.get("gpu_memory") or {}).get("size_in_gigabytes")
            count = int(gpu.get("number_of_gpus") or 0)
            for spot in (False, True):
                price = t.get("spot_price") if spot else t.get("price_per_hour")
                if price in (None, "", 0, "0"):
                    continue
                for loc in locations:
                    if self.config.get("regions") and loc not in self.config["regions"]:
                        continue
                    ok = name in stock.get((loc, spot), set())
                    rows.append(gpu_row(name, loc, float(price), (t.get("cpu") or {}).get("number_of_cores", 0),
                                        (t.get("memory") or {}).get("size_in_gigabytes", 0), gpu_name, count,
                                        spot=spot, gpu_memory_gb=(float(gpu_mem) / count if gpu_mem and count else None),
                                        availability=_AVAILABLE if ok else _NOT_AVAILABLE))
        return rows

    def _get_or_create_script(self, name: str, script: str) -> str:
        """A startup script with exactly this content is reused (they are account-level objects;
        one per launch would pile up), as the reference's ``get_or_create_startup_scrpit``."""
        r = check_response(self.http.get(f"{self.API}/scripts", headers=self._h()), "datacrunch scripts")
        for sc in r.json() or []:
            if sc.get("script") == script:
                return sc["id"]
        r = check_response(self.http.post(f"{self.API}/scripts", headers=self._h(), json={"name": name, "script": script}),
                           "datacrunch script")
        return r.json() if isinstance(r.json(), str) else r.json().get("id")

    def _get_or_create_keys(self, cfg) -> List[str]:
        """Account SSH keys matched by fingerprint (datacrunch/api_client.py ``get_or_create_ssh_key``)."""
        r = check_response(self.http.get(f"{self.API}/sshkeys", headers=self._h()), "datacrunch ssh keys")
        have = {}
        for k in r.json() or []:
            try:
                have[ssh_key_fingerprint(k.get("key", ""))] = k["id"]
            except (ValueError, IndexError):
                continue
        ids = []
        for pk in cfg.get_public_keys():
            fp = ssh_key_fingerprint(pk)
            if fp not in have:
                k = check_response(self.http.post(f"{self.API}/sshkeys", headers=self._h(),
                                                  json={"name": f"dstack-{cfg.instance_name}.key", "key": pk.strip()}),
                                   "datacrunch ssh key")
                have[fp] = k.json() if isinstance(k.json(), str) else k.json().get("id")
            ids.append(have[fp])
        return list(dict.fromkeys(ids))

    def _launch(self, offer, cfg):
        script_id = self._get_or_create_script(
            f"dstack-{cfg.instance_name}.sh",
            "#!/bin/bash\ncloud-init single --name runcmd || true\n" + _runcmd_script(cloud_init(cfg)))
        keys = self._get_or_create_keys(cfg)
        body = {"instance_type": offer.instance.name, "image": "ubuntu-22.04", "hostname": cfg.instance_name,
                "description": cfg.instance_name, "ssh_key_ids": keys, "location_code": offer.region,
                "startup_script_id": script_id, "is_spot": offer.instance.resources.spot,
                "os_volume": {"name": "os", "size": offer.instance.resources.disk.size_mib // 1024}}
        r = self.http.post(f"{self.API}/instances", headers=self._h(), json=body)
        if r.status_code == 400 and "not available" in r.text.lower():
            raise NoCapacityError(f"datacrunch: {offer.instance.name} not available in {offer.region}")
        check_response(r, "datacrunch deploy")
        iid = r.text.strip().strip('"')
        return iid, None, None

    def _describe(self, instance_id, region, backend_data):
        r = self.http.get(f"{self.API}/instances/{instance_id}", headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        d = check_response(r, "datacrunch get").json()
        return {"status": d.get("status"), "hostname": d.get("ip")}

    def _terminate(self, instance_id, region, backend_data):
        check_response(self.http.put(f"{self.API}/instances", headers=self._h(),
                                     json={"action": "delete", "id": instance_id}), "datacrunch delete")


class NebiusCompute(VMCompute):
    """Nebius AI cloud REST gateway (the reference's nebius backend).  Credentials: a service-account
    authorized key (``service_account`` creds: the key JSON with ``id``, ``service_account_id`` and
    ``private_key``), exchanged for short-lived IAM tokens with a PS256-signed JWT and cached until
    shortly before expiry; or a pre-issued IAM token."""

    TYPE = BackendType.NEBIUS
    API = "https://compute.api.nebius.cloud/compute/v1"
    IAM_TOKENS = "https://iam.api.nebius.cloud/iam/v1/tokens"

    def __init__(self, config, auth, client=None):
        super().__init__(config, auth, client)
        self._token = OAuthToken(self._exchange_sa_key)

    def _sa_key(self) -> Optional[dict]:
        import json

        data = self.auth.get("data")
        if not data:
            return None
        try:
            key = json.loads(data)
        except ValueError as e:
            raise BackendAuthError(f"nebius service account key is not JSON: {e}") from None
        if not all(k in key for k in ("id", "service_account_id", "private_key")):
            raise BackendAuthError("nebius service account key needs id, service_account_id and private_key")
        return key

    def _exchange_sa_key(self):
        import json
        import time as _time

        from dstack_amd.core.backends.clouds.common import b64url, rsa_sha256_sign

        key = self._sa_key()
        now = int(_time.time())
        header = {"typ": "JWT", "alg": "PS256", "kid": key["id"]}
        claims = {"aud": self.IAM_TOKENS, "iss": key["service_account_id"], "iat": now, "exp": now + 3600}
        signing_input = f"{b64url(json.dumps(header).encode())}.{b64url(json.dumps(claims).encode())}"
        sig = rsa_sha256_sign(key["private_key"], signing_input.encode(), pss=True)
        r = self.http.post(self.IAM_TOKENS, json={"jwt": f"{signing_input}.{b64url(sig)}"})
        if r.status_code in (400, 401, 403):
            raise BackendAuthError(f"nebius token exchange: {r.status_code} {r.text[:200]}")
        d = check_response(r, "nebius token exchange").json()
        return d["iamToken"], 3600

    def _h(self):
        static = self.auth.get("iam_token") or self.auth.get("token")
        return {"Authorization": f"Bearer {static or self._token.get()}"}

    def check_credentials(self) -> None:
        check_response(self.http.get(f"{self.API}/instances", params={"folderId": self.config.get("folder_id"),
                                                                      "pageSize": 1}, headers=self._h()),
                       "nebius instances")

    def _launch(self, offer, cfg):
        res = offer.instance.resources
        body = {"folderId": self.config.get("folder_id"), "name": cfg.instance_name, "zoneId": offer.region,
                "platformId": offer.instance.name.split(":")[0],
                "resourcesSpec": {"cores": res.cpus, "memory": res.memory_mib * 2**20, "gpus": len(res.gpus)},
                "metadata": {"user-data": cloud_init(cfg)},
                "bootDiskSpec": {"diskSpec": {"size": res.disk.size_mib * 2**20,
                                              "imageId": self.config.get("image_id", "ubuntu-22-04-lts-gpu")}},
                "networkInterfaceSpecs": [{"subnetId": self.config.get("subnet_id"),
                                           "primaryV4AddressSpec": {"oneToOneNatSpec": {"ipVersion": "IPV4"}}}]}
        r = check_response(self.http.post(f"{self.API}/instances", headers=self._h(), json=body), "nebius create")
        return r.json()["metadata"]["instanceId"], None, None

    def _describe(self, instance_id, region, backend_data):
        r = self.http.get(f"{self.API}/instances/{instance_id}", headers=self._h())
        if r.status_code == 404:
            return {"status": "terminated"}
        d = check_response(r, "nebius get").json()
        nic = (d.get("networkInterfaces") or [{}])[0]
        nat = nic.get("primaryV4Address", {}).get("oneToOneNat", {}).get("address")
        return {"status": d.get("status", "").lower(), "hostname": nat,
                "internal_ip": nic.get("primaryV4Address", {}).get("address")}

    def _terminate(self, instance_id, region, backend_data):
        r = self.http.delete(f"{self.API}/instances/{instance_id}", headers=self._h())
        if r.status_code != 404:
            check_response(r, "nebius delete")


def _runcmd_script(user_data: str) -> str:
    """Extract the runcmd lines of our cloud-config as a bash script (for clouds with plain
    startup scripts)."""
    import json

    out = []
    in_run = False
    for line in user_data.splitlines():
        if line.startswith("runcmd:"):
            in_run = True
            continue
        if in_run and line.startswith("  - "):
            out.append(json.loads(line[4:]))
        elif in_run:
            break
    return "\n".join(out) + "\n"


def eval_json(s: Optional[str]) -> Optional[Dict]:
    import json

    return json.loads(s) if s else None
