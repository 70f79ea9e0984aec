"""Container clouds: the job runs directly in a cloud container with ``dstack-runner`` as its
entrypoint (no shim) — reference: ``C/backends/runpod/compute.py:40-251`` (GraphQL),
``C/backends/vastai/compute.py`` and ``C/backends/kubernetes/compute.py:56-360``.

RunPod is the AMD MI300X container path; Kubernetes requests ``amd.com/gpu`` (ROCm device plugin)
and reaches pods through one SSH jump pod per backend (NodePort), as in the reference.
"""

from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Tuple

import httpx
import yaml

from dstack_amd.core.backends.base import Compute, DSTACK_RUNNER_SSH_PORT
from dstack_amd.core.backends.catalog import CatalogRow, gpu_row
from dstack_amd.core.backends.clouds.common import (
    CatalogOffers,
    check_response,
    container_commands,
    install_catalog_timeout,
)
from dstack_amd.core.errors import BackendAuthError, ComputeError, NoCapacityError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.gpus import normalize_gpu_name
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceOfferWithAvailability,
    SSHConnectionParams,
)
from dstack_amd.core.models.runs import Job, JobProvisioningData, Requirements, Run
from dstack_amd.core.models.volumes import Volume, VolumeProvisioningData

from dstack_amd.core.models.images import DEFAULT_ROCM_IMAGE  # noqa: E402 - one gfx950-capable image


def _job_image(job: Job) -> str:
    return job.job_spec.image_name or DEFAULT_ROCM_IMAGE


def _entrypoint(keys: List[str]) -> str:
    return " && ".join(container_commands(keys))


class ContainerCompute(CatalogOffers, Compute):
    def __init__(self, config: Dict, auth: Dict, client: Optional[httpx.Client] = None):
        super().__init__()
        self.config, self.auth = config or {}, auth or {}
        self.http = install_catalog_timeout(client or httpx.Client(timeout=60))


# ---------------------------------------------------------------------------------------------
class RunpodCompute(ContainerCompute):
    TYPE = BackendType.RUNPOD
    API = "https://api.runpod.io/graphql"
    CONFIGURABLE_DISK = (10.0, None)
    GPU_COUNTS = (1, 2, 4, 8)
    GPU_TYPE_IDS = {"MI300X": "AMD Instinct MI300X OAM"}
    CATALOG_QUERY = (
        "query { gpuTypes { id displayName memoryInGb maxGpuCount securePrice secureSpotPrice "
        "lowestPrice(input: {gpuCount: 1}) { minVcpu minMemory } } "
        "dataCenters { id listed gpuAvailability { gpuTypeId available stockStatus } } }"
    )

    def check_credentials(self) -> None:
        try:
            self._gql("query { myself { id } }")
        except ComputeError as e:
            if any(w in str(e).lower() for w in ("unauthorized", "api key", "forbidden", "authenticated")):
                raise BackendAuthError(str(e)) from None
            raise

    def _fetch_catalog(self) -> List[CatalogRow]:
        """GPU types (secure-cloud on-demand and spot price per GPU, vCPU / RAM per GPU) x data
        centres' per-type stock; instance name ``<n>x-<GPU>`` as in the offline catalog."""
        d = self._gql(self.CATALOG_QUERY)
        types = {t["id"]: t for t in d.get("gpuTypes") or []}
        wanted = self.config.get("regions")
        rows = []
        for dc in d.get("dataCenters") or []:
            if dc.get("listed") is False or (wanted and dc.get("id") not in wanted):
                continue
            for ga in dc.get("gpuAvailability") or []:
                t = types.get(ga.get("gpuTypeId"))
                if not t:
                    continue
                name = normalize_gpu_name(t.get("displayName") or t["id"])
                self.GPU_TYPE_IDS = {**self.GPU_TYPE_IDS, name: t["id"]}
                low = t.get("lowestPrice") or {}
                ok = bool(ga.get("available")) or (ga.get("stockStatus") or "").lower() in ("high", "medium", "low")
                for n in self.GPU_COUNTS:
                    if n > int(t.get("maxGpuCount") or 8):
                        break
                    for spot, price in ((False, t.get("securePrice")), (True, t.get("secureSpotPrice"))):
                        if not price:
                            continue
                        rows.append(gpu_row(f"{n}x-{name}", dc["id"], n * float(price),
                                            n * int(low.get("minVcpu") or 8), n * int(low.get("minMemory") or 32),
                                            name, n, spot=spot, gpu_memory_gb=t.get("memoryInGb"),
                                            availability=InstanceAvailability.AVAILABLE if ok
                                            else InstanceAvailability.NOT_AVAILABLE))
        return rows

    def _gql(self, query: str, variables: Optional[dict] = None) -> dict:
        r = self.http.post(self.API, params={"api_key": self.auth.get("api_key", "")},
                           json={"query": query, "variables": variables or {}})
        d = check_response(r, "runpod graphql").json()
        if d.get("errors"):
            msg = "; ".join(e.get("message", "") for e in d["errors"])
            if "no longer any instances available" in msg.lower() or "not enough" in msg.lower():
                raise NoCapacityError(f"runpod: {msg}")
            raise ComputeError(f"runpod: {msg}")
        return d["data"]

    def run_job(self, run: Run, job: Job, instance_offer: InstanceOfferWithAvailability, project_ssh_public_key: str,
                project_ssh_private_key: str, volumes: List[Volume]) -> JobProvisioningData:
        res = instance_offer.instance.resources
        keys = [project_ssh_public_key.strip()] + ([run.run_spec.ssh_key_pub.strip()] if run.run_spec.ssh_key_pub else [])
        gpu_type = self.GPU_TYPE_IDS.get(res.gpus[0].name, res.gpus[0].name) if res.gpus else None
        inp = {
            "name": f"{run.run_spec.run_name}-{job.job_spec.job_num}", "imageName": _job_image(job),
            "gpuTypeId": gpu_type, "gpuCount": len(res.gpus), "cloudType": "SECURE" if not res.spot else "COMMUNITY",
            "containerDiskInGb": max(10, res.disk.size_mib // 1024), "volumeInGb": 0, "minVcpuCount": res.cpus,
            "minMemoryInGb": res.memory_mib // 1024, "dataCenterId": instance_offer.region,
            "dockerArgs": f"bash -c {json.dumps(_entrypoint(keys))}",
            "ports": f"{DSTACK_RUNNER_SSH_PORT}/tcp", "supportPublicIp": True,
            "env": [{"key": "DSTACK_RUNNER_SSH", "value": "1"}],
        }
        if volumes:
            inp["networkVolumeId"] = volumes[0].volume_id
            inp["volumeMountPath"] = "/workspace"
        mutation = "mutation($input: PodFindAndDeployOnDemandInput) { podFindAndDeployOnDemand(input: $input) " \
                   "{ id machineId } }"
        if res.spot:
            mutation = "mutation($input: PodRentInterruptableInput!) { podRentInterruptable(input: $input) " \
                       "{ id machineId } }"
            inp["bidPerGpu"] = instance_offer.price / max(1, len(res.gpus))
        data = self._gql(mutation, {"input": inp})
        pod = data.get("podFindAndDeployOnDemand") or data.get("podRentInterruptable")
        return JobProvisioningData(
            backend=self.TYPE, instance_type=instance_offer.instance, instance_id=pod["id"], hostname=None,
            region=instance_offer.region, price=instance_offer.price, username="root", ssh_port=None,
            dockerized=False, backend_data=json.dumps({"machine_id": pod.get("machineId")}))

    def update_provisioning_data(self, provisioning_data: JobProvisioningData, project_ssh_public_key: str = "",
                                 project_ssh_private_key: str = "") -> None:
        q = "query($id: String!) { pod(input: {podId: $id}) { id runtime { ports { ip isIpPublic privatePort " \
            "publicPort type } } } }"
        pod = self._gql(q, {"id": provisioning_data.instance_id}).get("pod") or {}
        for p in ((pod.get("runtime") or {}).get("ports") or []):
            if p.get("privatePort") == DSTACK_RUNNER_SSH_PORT and p.get("isIpPublic"):
                provisioning_data.hostname = p["ip"]
                provisioning_data.ssh_port = p["publicPort"]

    def terminate_instance(self, instance_id: str, region: str, backend_data: Optional[str] = None) -> None:
        try:
            self._gql("mutation($id: String!) { podTerminate(input: {podId: $id}) }", {"id": instance_id})
        except ComputeError as e:
            if "not found" not in str(e).lower():
                raise

    def create_volume(self, volume: Volume) -> VolumeProvisioningData:
        conf = volume.configuration
        q = "mutation($input: CreateNetworkVolumeInput!) { createNetworkVolume(input: $input) { id size } }"
        d = self._gql(q, {"input": {"name": volume.name, "size": int(conf.size or 100), "dataCenterId": conf.region}})
        v = d["createNetworkVolume"]
        return VolumeProvisioningData(backend=self.TYPE, volume_id=v["id"], size_gb=int(v["size"]),
                                      price=0.07 * int(v["size"]) / 730, attachable=False, detachable=False)

    def register_volume(self, volume: Volume) -> VolumeProvisioningData:
        d = self._gql("query { myself { networkVolumes { id name size dataCenterId } } }")
        for v in d["myself"]["networkVolumes"]:
            if v["id"] == volume.configuration.volume_id:
                return VolumeProvisioningData(backend=self.TYPE, volume_id=v["id"], size_gb=int(v["size"]),
                                              attachable=False, detachable=False)
        raise ComputeError(f"runpod volume {volume.configuration.volume_id} not found")

    def delete_volume(self, volume: Volume) -> None:
        self._gql("mutation($id: String!) { deleteNetworkVolume(input: {id: $id}) }", {"id": volume.volume_id})


# ---------------------------------------------------------------------------------------------
class VastAICompute(ContainerCompute):
    TYPE = BackendType.VASTAI
    API = "https://console.vast.ai/api/v0"

    def _h(self):
        return {"Authorization": f"Bearer {self.auth.get('api_key', '')}"}

    def check_credentials(self) -> None:
        check_response(self.http.get(f"{self.API}/users/current/", headers=self._h()), "vastai user")

    def _fetch_catalog(self) -> List[CatalogRow]:
        """Live marketplace asks (``/bundles``): one row per rentable offer, named by its ask id."""
        r = check_response(self.http.post(f"{self.API}/bundles/", headers=self._h(), json={
            "rentable": {"eq": True}, "rented": {"eq": False}, "order": [["dph_total", "asc"]], "limit": 500}),
            "vastai bundles")
        rows = []
        for a in r.json().get("offers") or []:
            n = int(a.get("num_gpus") or 0)
            rows.append(gpu_row(str(a["id"]), str(a.get("geolocation") or "any"), float(a["dph_total"]),
                                int(a.get("cpu_cores_effective") or 1), float(a.get("cpu_ram") or 0) / 1024,
                                a.get("gpu_name") or None, n, disk_gb=float(a.get("disk_space") or 100),
                                gpu_memory_gb=float(a.get("gpu_ram") or 0) / 1024 or None,
                                availability=InstanceAvailability.AVAILABLE))
        return rows

    def run_job(self, run, job, instance_offer, project_ssh_public_key, project_ssh_private_key, volumes):
        keys = [project_ssh_public_key.strip()] + ([run.run_spec.ssh_key_pub.strip()] if run.run_spec.ssh_key_pub else [])
        body = {"client_id": "me", "image": _job_image(job), "disk": instance_offer.instance.resources.disk.size_mib // 1024,
                "label": f"{run.run_spec.run_name}-{job.job_spec.job_num}", "onstart": _entrypoint(keys),
                "runtype": "args", "env": {f"-p {DSTACK_RUNNER_SSH_PORT}:{DSTACK_RUNNER_SSH_PORT}": "1"}}
        r = check_response(self.http.put(f"{self.API}/asks/{instance_offer.instance.name}/", headers=self._h(),
                                         json=body), "vastai rent")
        d = r.json()
        if not d.get("success"):
            raise NoCapacityError(f"vastai: {d}")
        return JobProvisioningData(backend=self.TYPE, instance_type=instance_offer.instance,
                                   instance_id=str(d["new_contract"]), hostname=None, region=instance_offer.region,
                                   price=instance_offer.price, username="root", ssh_port=None, dockerized=False)

    def update_provisioning_data(self, provisioning_data, project_ssh_public_key="", project_ssh_private_key=""):
        r = check_response(self.http.get(f"{self.API}/instances/{provisioning_data.instance_id}/",
                                         headers=self._h()), "vastai get")
        inst = r.json().get("instances") or {}
        ports = (inst.get("ports") or {}).get(f"{DSTACK_RUNNER_SSH_PORT}/tcp") or []
        if inst.get("actual_status") == "running" and ports:
            provisioning_data.hostname = inst.get("public_ipaddr", "").strip()
            provisioning_data.ssh_port = int(ports[0]["HostPort"])

    def terminate_instance(self, instance_id, region, backend_data=None):
        r = self.http.delete(f"{self.API}/instances/{instance_id}/", headers=self._h())
        if r.status_code != 404:
            check_response(r, "vastai delete")


# ---------------------------------------------------------------------------------------------
class KubernetesCompute(ContainerCompute):
    """Pods with ``amd.com/gpu`` limits; SSH through a per-backend jump pod (NodePort service)."""

    TYPE = BackendType.KUBERNETES
    NAMESPACE = "default"

    def __init__(self, config, auth, client=None):
        super().__init__(config, auth, client)
        self._kube = self._load_kubeconfig()
        self.namespace = self.config.get("namespace", self.NAMESPACE)

    def _load_kubeconfig(self) -> dict:
        kc = self.config.get("kubeconfig") or {}
        data = kc.get("data")
        if data is None and kc.get("filename"):
            with open(os.path.expanduser(kc["filename"])) as f:
                data = f.read()
        if not data:
            return {"server": self.config.get("api_url", "https://kubernetes.default.svc"), "token": self.auth.get("token")}
        d = yaml.safe_load(data)
        ctx_name = d.get("current-context")
        ctx = next((c["context"] for c in d.get("contexts", []) if c["name"] == ctx_name), d["contexts"][0]["context"])
        cluster = next(c["cluster"] for c in d["clusters"] if c["name"] == ctx["cluster"])
        user = next(u["user"] for u in d["users"] if u["name"] == ctx["user"])
        return {"server": cluster["server"], "ca": cluster.get("certificate-authority-data"),
                "token": user.get("token"), "cert": user.get("client-certificate-data"),
                "key": user.get("client-key-data")}

    def _h(self):
        return {"Authorization": f"Bearer {self._kube['token']}"} if self._kube.get("token") else {}

    def _url(self, path: str) -> str:
        return self._kube["server"].rstrip("/") + path

    def check_credentials(self) -> None:
        check_response(self.http.get(self._url(f"/api/v1/namespaces/{self.NAMESPACE}"), headers=self._h()),
                       "kubernetes namespace")

    def get_offers(self, requirements: Optional[Requirements] = None) -> List[InstanceOfferWithAvailability]:
        """One offer per node (allocatable CPU/memory/``amd.com/gpu``)."""
        from dstack_amd.core.backends.base import offer_matches
        from dstack_amd.core.models.instances import Disk, Gpu, InstanceType, Resources

        try:
            r = self.http.get(self._url("/api/v1/nodes"), headers=self._h())
            nodes = r.json().get("items", []) if r.status_code == 200 else []
        except httpx.HTTPError:
            nodes = []
        out = []
        for n in nodes:
            alloc = n.get("status", {}).get("allocatable", {})
            labels = n.get("metadata", {}).get("labels", {})
            res = Resources(cpus=_cpu(alloc.get("cpu", "1")), memory_mib=_mem_mib(alloc.get("memory", "0")),
                            gpus=gpus_from_node_labels(labels, alloc), spot=False,
                            disk=Disk(size_mib=_mem_mib(alloc.get("ephemeral-storage", "100Gi"))))
            o = InstanceOfferWithAvailability(backend=self.TYPE, instance=InstanceType(
                name=n["metadata"]["name"], resources=res), region=self.namespace, price=0.0,
                availability=InstanceAvailability.AVAILABLE)
            if offer_matches(o, requirements):
                out.append(o)
        return out

    def _ensure_jump_pod(self, project_ssh_public_key: str) -> Tuple[str, int]:
        name = "dstack-ssh-jump"
        r = self.http.get(self._url(f"/api/v1/namespaces/{self.namespace}/services/{name}"), headers=self._h())
        if r.status_code == 404:
            pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": {"app": name}},
                   "spec": {"containers": [{"name": "sshd", "image": "linuxserver/openssh-server:latest",
                                            "env": [{"name": "PUBLIC_KEY", "value": project_ssh_public_key},
                                                    {"name": "USER_NAME", "value": "root"}],
                                            "ports": [{"containerPort": 2222}]}]}}
            check_response(self.http.post(self._url(f"/api/v1/namespaces/{self.namespace}/pods"), headers=self._h(),
                                          json=pod), "k8s jump pod")
            svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name},
                   "spec": {"type": "NodePort", "selector": {"app": name}, "ports": [{"port": 22, "targetPort": 2222}]}}
            r = check_response(self.http.post(self._url(f"/api/v1/namespaces/{self.namespace}/services"),
                                              headers=self._h(), json=svc), "k8s jump service")
        port = r.json()["spec"]["ports"][0]["nodePort"]
        host = self.config.get("networking", {}).get("ssh_host") or httpx.URL(self._kube["server"]).host
        return host, int(port)

    def run_job(self, run, job, instance_offer, project_ssh_public_key, project_ssh_private_key, volumes):
        keys = [project_ssh_public_key.strip()] + ([run.run_spec.ssh_key_pub.strip()] if run.run_spec.ssh_key_pub else [])
        res = instance_offer.instance.resources
        name = f"{run.run_spec.run_name}-{job.job_spec.job_num}-{job.job_spec.replica_num}"[:60]
        limits = {"cpu": str(res.cpus), "memory": f"{res.memory_mib}Mi"}
        if res.gpus:
            limits["amd.com/gpu"] = str(len(res.gpus))
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": {"app.kubernetes.io/name": name}},
               "spec": {"restartPolicy": "Never", "nodeName": instance_offer.instance.name,
                        "containers": [{"name": "job", "image": _job_image(job), "command": ["/bin/bash", "-c"],
                                        "args": [_entrypoint(keys)], "ports": [{"containerPort": DSTACK_RUNNER_SSH_PORT}],
                                        "resources": {"limits": limits, "requests": limits},
                                        "securityContext": {"capabilities": {"add": ["SYS_PTRACE", "IPC_LOCK"]}},
                                        "volumeMounts": [{"name": "shm", "mountPath": "/dev/shm"}]}],
                        "volumes": [{"name": "shm", "emptyDir": {"medium": "Memory"}}]}}
        check_response(self.http.post(self._url(f"/api/v1/namespaces/{self.namespace}/pods"), headers=self._h(),
                                      json=pod), "k8s create pod")
        svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name},
               "spec": {"type": "ClusterIP", "selector": {"app.kubernetes.io/name": name},
                        "ports": [{"port": DSTACK_RUNNER_SSH_PORT}]}}
        check_response(self.http.post(self._url(f"/api/v1/namespaces/{self.namespace}/services"), headers=self._h(),
                                      json=svc), "k8s create service")
        jump_host, jump_port = self._ensure_jump_pod(project_ssh_public_key)
        return JobProvisioningData(
            backend=self.TYPE, instance_type=instance_offer.instance, instance_id=name, hostname=None,
            region=self.namespace, price=0.0, username="root", ssh_port=DSTACK_RUNNER_SSH_PORT, dockerized=False,
            ssh_proxy=SSHConnectionParams(hostname=jump_host, username="root", port=jump_port))

    def update_provisioning_data(self, provisioning_data, project_ssh_public_key="", project_ssh_private_key=""):
        r = check_response(self.http.get(self._url(f"/api/v1/namespaces/{self.namespace}/services/"
                                                    f"{provisioning_data.instance_id}"), headers=self._h()), "k8s svc")
        ip = r.json().get("spec", {}).get("clusterIP")
        p = self.http.get(self._url(f"/api/v1/namespaces/{self.namespace}/pods/{provisioning_data.instance_id}"),
                          headers=self._h()).json()
        if p.get("status", {}).get("phase") == "Running" and ip:
            provisioning_data.hostname = ip
            provisioning_data.internal_ip = p["status"].get("podIP")

    def terminate_instance(self, instance_id, region, backend_data=None):
        for kind in ("services", "pods"):
            r = self.http.delete(self._url(f"/api/v1/namespaces/{self.namespace}/{kind}/{instance_id}"),
                                 headers=self._h())
            if r.status_code not in (200, 202, 404):
                check_response(r, f"k8s delete {kind}")

    # ---- gateway: pod + LoadBalancer service (reference ``C/backends/kubernetes/compute.py:221-310``) ----
    def create_gateway(self, configuration):
        """A ``ubuntu:22.04`` pod running sshd, nginx and the versioned gateway app, exposed by a
        ``LoadBalancer`` service on 22/80/443.  Needs a cluster with load-balancer support: without
        an external address after the wait the pod and service are removed and creation fails."""
        from dstack_amd.core.models.gateways import GatewayProvisioningData
        from dstack_amd.proxy.gateway.packaging import container_commands

        name = configuration.instance_name.lower().replace("_", "-")[:50]
        ns = self.namespace
        cmds = container_commands(configuration.ssh_key_pub)
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": name, "labels": {"app.kubernetes.io/name": name, "dstack/role": "gateway"}},
               "spec": {"containers": [{"name": "gateway", "image": "ubuntu:22.04", "command": ["/bin/sh"],
                                        "args": ["-c", " && ".join(cmds)],
                                        "ports": [{"containerPort": p} for p in (22, 80, 443)]}]}}
        check_response(self.http.post(self._url(f"/api/v1/namespaces/{ns}/pods"), headers=self._h(), json=pod),
                       "k8s gateway pod")
        svc_name = f"{name}-service"
        svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": svc_name},
               "spec": {"type": "LoadBalancer", "selector": {"app.kubernetes.io/name": name},
                        "ports": [{"name": n, "port": p, "targetPort": p}
                                  for n, p in (("ssh", 22), ("http", 80), ("https", 443))]}}
        check_response(self.http.post(self._url(f"/api/v1/namespaces/{ns}/services"), headers=self._h(), json=svc),
                       "k8s gateway service")
        host = None
        for _ in range(int(self.config.get("gateway_lb_wait_tries", 60))):
            r = self.http.get(self._url(f"/api/v1/namespaces/{ns}/services/{svc_name}"), headers=self._h())
            if r.status_code == 200:
                ing = (r.json().get("status", {}).get("loadBalancer", {}).get("ingress") or [{}])[0]
                host = ing.get("hostname") or ing.get("ip")
                if host:
                    break
            time.sleep(float(self.config.get("gateway_lb_wait_s", 5)))
        if not host:
            self.terminate_gateway(name, configuration)
            raise ComputeError("the gateway's LoadBalancer service got no external address "
                               "(does the cluster support LoadBalancer services?)")
        return GatewayProvisioningData(instance_id=name, ip_address=host, region=ns,
                                       backend_data=json.dumps({"ssh_user": "root", "service": svc_name}))

    def terminate_gateway(self, instance_id, configuration, backend_data=None):
        svc = json.loads(backend_data or "{}").get("service", f"{instance_id}-service")
        for kind, n in (("services", svc), ("pods", instance_id)):
            r = self.http.delete(self._url(f"/api/v1/namespaces/{self.namespace}/{kind}/{n}"), headers=self._h())
            if r.status_code not in (200, 202, 404):
                check_response(r, f"k8s delete gateway {kind}")


# AMD GPU operator's node labeller: PCI device id -> catalog name (when product-name is absent)
_AMD_DEVICE_IDS = {"75a3": "MI355X", "75a0": "MI350X", "74a5": "MI325X", "74a1": "MI300X", "74a0": "MI300A",
                   "740c": "MI250X", "740f": "MI210", "738c": "MI100"}


def gpus_from_node_labels(labels: dict, allocatable: Optional[dict] = None):
    """The GPUs a Kubernetes node offers, from its device-plugin resources and node labels (reference
    ``C/backends/kubernetes/compute.py`` ``_get_gpus_from_node_labels``, which reads NVIDIA's GPU
    feature discovery labels only).

    AMD first: the count is the allocatable ``amd.com/gpu`` (or the ``amd.com/gpu.count`` label), the
    model the labeller's ``amd.com/gpu.product-name`` (``AMD_Instinct_MI300X_OAM``) or
    ``amd.com/gpu.device-id``, the memory ``amd.com/gpu.vram`` (``192G``) or the catalog's. NVIDIA:
    ``nvidia.com/gpu.count`` + ``nvidia.com/gpu.product`` (``A100-SXM4-80GB``), memory from
    ``nvidia.com/gpu.memory`` (MiB), the product's ``<n>GB`` suffix or the catalog. A node whose
    GPU model cannot be told offers no GPUs (it is not guessed)."""
    import re as _re

    from dstack_amd.core.models.gpus import convert_nvidia_gpu_name, gpu_info, normalize_gpu_name
    from dstack_amd.core.models.instances import Gpu

    allocatable = allocatable or {}
    amd_n = int(allocatable.get("amd.com/gpu") or labels.get("amd.com/gpu.count") or 0)
    if amd_n:
        product = labels.get("amd.com/gpu.product-name") or labels.get("beta.amd.com/gpu.product-name")
        name = normalize_gpu_name(product.replace("_", " ")) if product else None
        if not name:
            dev = str(labels.get("amd.com/gpu.device-id") or labels.get("beta.amd.com/gpu.device-id") or "").lower()
            name = _AMD_DEVICE_IDS.get(dev.removeprefix("0x"))
        if not name:
            return []
        vram = _re.fullmatch(r"(\d+)\s*([GM])i?B?", str(labels.get("amd.com/gpu.vram") or ""), _re.I)
        if vram:
            mib = int(vram.group(1)) * (1024 if vram.group(2).upper() == "G" else 1)
        else:
            info = gpu_info(name)
            mib = int(info.memory_gb * 1024) if info else 0
        return [Gpu(name=name, memory_mib=mib, vendor="amd") for _ in range(amd_n)]
    nv_n = int(labels.get("nvidia.com/gpu.count") or allocatable.get("nvidia.com/gpu") or 0)
    product = labels.get("nvidia.com/gpu.product")
    if not nv_n or not product:
        return []
    name = convert_nvidia_gpu_name(product.split("-")[0].replace("NVIDIA", "").strip() or product)
    if labels.get("nvidia.com/gpu.memory"):
        mib = int(labels["nvidia.com/gpu.memory"])
    else:
        m = _re.search(r"(\d+)GB", product, _re.I)
        info = gpu_info(name)
        mib = int(m.group(1)) * 1024 if m else (int(info.memory_gb * 1024) if info else 0)
    return [Gpu(name=name, memory_mib=mib, vendor="nvidia") for _ in range(nv_n)]


def _cpu(v: str) -> int:
    return max(1, int(float(v[:-1]) / 1000) if v.endswith("m") else int(float(v)))


def _mem_mib(v: str) -> int:
    units = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024, "Ti": 1024 * 1024, "K": 1 / 1024, "M": 1, "G": 1024}
    for u, m in units.items():
        if v.endswith(u):
            return int(float(v[: -len(u)]) * m)
    return int(float(v) / 2**20)
