"""Offer catalog layers (catalog.py): built-in table, downloaded offline catalog, per-backend live
listings with a TTL / stale-tolerant cache, and the reference's disk-size rules
(``C/backends/base/offers.py:18-175``).  Live listings run against mock transports shaped like each
provider's public API."""

import io
import json
import time
import urllib.parse
import zipfile
import xml.etree.ElementTree as ET

import httpx
import pytest

from dstack_amd.core.backends import catalog
from dstack_amd.core.backends.catalog import (
    CatalogRow,
    OfflineCatalog,
    OnlineCache,
    catalog_offers,
    dump_catalog_csv,
    get_catalog_offers,
    gpu_row,
    parse_catalog_csv,
)
from dstack_amd.core.backends.clouds import compute_class
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceAvailability as IA
from dstack_amd.core.models.resources import ResourcesSpec
from dstack_amd.core.models.runs import Requirements


def _req(spot=None, **res):
    return Requirements(resources=ResourcesSpec.model_validate(res), spot=spot)


def _client(handler):
    return httpx.Client(transport=httpx.MockTransport(handler))


@pytest.fixture
def live(monkeypatch, tmp_path):
    """Live listings on, cache in a fresh directory."""
    monkeypatch.delenv("DSTACK_CATALOG_OFFLINE_ONLY", raising=False)
    monkeypatch.setenv("DSTACK_CATALOG_CACHE_DIR", str(tmp_path / "cache"))
    monkeypatch.delenv("DSTACK_CATALOG_URL", raising=False)
    monkeypatch.delenv("DSTACK_CATALOG_PATH", raising=False)
    catalog.reset_catalog_state()
    yield tmp_path
    catalog.reset_catalog_state()


# ---- rows -> offers ---------------------------------------------------------------------------
def test_builtin_rows_and_disk_rules():
    # bare metal has a fixed local disk: kept as is, and must fit the requested range
    vultr = catalog_offers(BackendType.VULTR, None, _req(gpu="MI355X:8"))
    assert vultr and all(o.instance.resources.disk.size_mib == 15000 * 1024 for o in vultr)
    assert not catalog_offers(BackendType.VULTR, None, _req(gpu="MI355X:8", disk="200GB"))
    # configurable disks take the requested minimum, clamped to the cloud's range
    aws = compute_class(BackendType.AWS)({"regions": ["us-east-1"]}, {})
    (o,) = [o for o in aws.get_offers(_req(gpu="H100:8", disk="500GB..", spot=False))]
    assert o.instance.resources.disk.size_mib == 500 * 1024
    assert not aws.get_offers(_req(gpu="H100:8", disk="20000GB.."))
    # regions filter and GPU facts from the GPU table
    (ewr,) = catalog_offers(BackendType.VULTR, ["ewr"], _req(gpu="MI355X:8"))
    g = ewr.instance.resources.gpus[0]
    assert (g.name, g.memory_mib, g.vendor.value) == ("MI355X", 288 * 1024, "amd")


def test_csv_round_trip():
    rows = [gpu_row("vbm-8-mi355x", "sjc", 19.5, 256, 3072, "mi355x", 8, disk_gb=15000),
            gpu_row("c6i.xlarge", "us-east-1", 0.05, 4, 8, None, 0, spot=True)]
    back = parse_catalog_csv(dump_catalog_csv(rows))
    assert back == rows
    assert back[0].gpu_name == "MI355X" and back[0].gpu_memory_gb == 288 and back[1].disk_gb is None


def _zip(files):
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        for name, text in files.items():
            z.writestr(name, text)
    return buf.getvalue()


def test_offline_catalog_download_ttl_and_stale_copy(live, monkeypatch):
    csv_text = dump_catalog_csv([gpu_row("vbm-8-mi355x", "sjc", 19.5, 256, 3072, "MI355X", 8, disk_gb=15000)])
    calls = []

    def fetch(url):
        calls.append(url)
        if len(calls) > 1:
            raise OSError("offline")
        return _zip({"vultr.csv": csv_text, "lambdalabs.csv": dump_catalog_csv([])})

    off = OfflineCatalog(url="https://catalog.example/v2/catalog.zip", ttl=3600, fetch=fetch)
    rows = off.rows(BackendType.VULTR)
    assert [r.location for r in rows] == ["sjc"]
    assert off.rows(BackendType.LAMBDA) == []
    assert off.rows(BackendType.AWS) is None  # provider missing -> built-in table
    off.rows(BackendType.VULTR)
    assert len(calls) == 1  # within the TTL: no second download
    # expired + download failing: the cached zip keeps serving
    off2 = OfflineCatalog(url="https://catalog.example/v2/catalog.zip", ttl=0.0, fetch=fetch)
    assert [r.location for r in off2.rows(BackendType.VULTR)] == ["sjc"]
    assert len(calls) == 2


def test_offline_catalog_from_path_feeds_offers(live, monkeypatch):
    d = live / "cat"
    d.mkdir()
    (d / "vultr.csv").write_text(dump_catalog_csv([
        gpu_row("vbm-8-mi355x", "sjc", 19.5, 256, 3072, "MI355X", 8, disk_gb=15000)]))
    monkeypatch.setenv("DSTACK_CATALOG_PATH", str(d))
    catalog.reset_catalog_state()
    offers = catalog_offers(BackendType.VULTR, None, _req(gpu="MI355X:8"))
    assert [(o.instance.name, o.region, o.price) for o in offers] == [("vbm-8-mi355x", "sjc", 19.5)]
    # backends absent from the downloaded catalog keep the built-in rows
    assert catalog_offers(BackendType.OCI, None, _req(gpu="MI355X:8"))


def test_online_cache_ttl_stale_and_disk(tmp_path):
    row = gpu_row("t", "r", 1.0, 1, 1, None, 0)
    n = {"calls": 0}

    def ok():
        n["calls"] += 1
        return [row]

    def boom():
        raise RuntimeError("api down")

    c = OnlineCache(ttl=60, max_stale=3600, directory=tmp_path)
    assert c.get("k", ok) == [row] and c.get("k", ok) == [row] and n["calls"] == 1
    # a new process (fresh memory) reads the persisted listing within the TTL
    c2 = OnlineCache(ttl=60, max_stale=3600, directory=tmp_path)
    assert c2.get("k", boom) == [row]
    # TTL expired and the refresh fails: stale rows within max_stale, then nothing
    c3 = OnlineCache(ttl=0, max_stale=3600, directory=tmp_path)
    assert c3.get("k", boom) == [row]
    c4 = OnlineCache(ttl=0, max_stale=0, directory=tmp_path)
    assert c4.get("k", boom) is None
    assert c4.get("other", boom) is None


def test_failed_live_listing_falls_back_to_offline(live):
    c = compute_class(BackendType.LAMBDA)({}, {"api_key": "k"}, _client(lambda r: httpx.Response(503)))
    offers = c.get_offers(_req(gpu="H100:8"))
    assert offers and offers[0].availability == IA.UNKNOWN  # the built-in row


def test_unreachable_listing_is_fetched_once_per_backoff(live, monkeypatch):
    """Negative caching: a listing that failed is not fetched again for the backoff period (cached
    or offline rows meanwhile), so an air-gapped server does not stall every plan on the API; and
    live listings run with the short catalog timeout, not the client's launch timeout."""
    timeouts = []

    def handler(r):
        timeouts.append(r.extensions.get("timeout"))
        raise httpx.ConnectError("unreachable")

    c = compute_class(BackendType.LAMBDA)({}, {"api_key": "k"}, _client(handler))
    for _ in range(3):
        assert c.get_offers(_req(gpu="H100:8"))  # the built-in rows
    assert len(timeouts) == 1
    assert timeouts[0]["connect"] == catalog.catalog_fetch_timeout() == 10.0
    # outside a catalog fetch the same client keeps its own timeout
    try:
        c.http.get("https://cloud.lambdalabs.com/api/v1/instances")
    except httpx.ConnectError:
        pass
    assert timeouts[-1]["connect"] != 10.0
    # after the backoff the listing is tried again
    monkeypatch.setattr(catalog._online, "failure_backoff", 0.0)
    c.get_offers(_req(gpu="H100:8"))
    assert len(timeouts) == 3


def test_online_cache_failure_backoff_serves_stale(tmp_path):
    row = gpu_row("t", "r", 1.0, 1, 1, None, 0)
    n = {"calls": 0}

    def boom():
        n["calls"] += 1
        raise RuntimeError("api down")

    c = OnlineCache(ttl=60, max_stale=3600, directory=tmp_path)
    c.get("k", lambda: [row])
    c._mem["k"] = (time.time() - 120, [row])  # expired, still within max_stale
    assert c.get("k", boom) == [row] and c.get("k", boom) == [row] and n["calls"] == 1


def test_offline_only_switch(live, monkeypatch):
    hits = []
    c = compute_class(BackendType.LAMBDA)({"offline_catalog": True}, {"api_key": "k"},
                                          _client(lambda r: hits.append(r) or httpx.Response(500)))
    assert c.get_offers(None) and not hits


# ---- live listings ------------------------------------------------------------------------------
def test_lambda_live_listing(live):
    def handler(req):
        assert req.url.path == "/api/v1/instance-types" and req.headers["authorization"] == "Bearer k"
        return httpx.Response(200, json={"data": {
            "gpu_8x_h100_sxm5": {"instance_type": {
                "name": "gpu_8x_h100_sxm5", "price_cents_per_hour": 2392, "gpu_description": "H100 (80 GB SXM5)",
                "specs": {"vcpus": 208, "memory_gib": 1800, "storage_gib": 22000, "gpus": 8}},
                "regions_with_capacity_available": [{"name": "us-west-2"}]},
            "cpu_4x_general": {"instance_type": {
                "name": "cpu_4x_general", "price_cents_per_hour": 20, "gpu_description": "",
                "specs": {"vcpus": 4, "memory_gib": 16, "storage_gib": 100, "gpus": 0}},
                "regions_with_capacity_available": []}}})

    c = compute_class(BackendType.LAMBDA)({"regions": ["us-west-2", "us-east-1"]}, {"api_key": "k"},
                                          _client(handler))
    offers = c.get_offers(_req(gpu="H100:8"))
    by_region = {o.region: o for o in offers}
    assert set(by_region) == {"us-west-2", "us-east-1"}
    assert by_region["us-west-2"].availability == IA.AVAILABLE and by_region["us-west-2"].price == 23.92
    assert by_region["us-east-1"].availability == IA.NOT_AVAILABLE
    res = by_region["us-west-2"].instance.resources
    assert res.disk.size_mib == 22000 * 1024 and res.gpus[0].memory_mib == 80 * 1024
    cpu = c.get_offers(_req(gpu=0))
    assert cpu and all(not o.instance.resources.gpus for o in cpu)


def test_vultr_live_listing(live):
    def handler(req):
        p = req.url.path
        if p == "/v2/plans":
            return httpx.Response(200, json={"plans": [
                {"id": "vcg-a100-12c-120g-80vram", "type": "vcg", "vcpu_count": 12, "ram": 122880, "disk": 1400,
                 "monthly_cost": 1750, "gpu_vram_gb": 80, "gpu_type": "NVIDIA_A100", "locations": ["ewr"]},
                {"id": "vcg-a100-1c-6g-4vram", "type": "vcg", "vcpu_count": 1, "ram": 6144, "disk": 70,
                 "monthly_cost": 90, "gpu_vram_gb": 4, "gpu_type": "NVIDIA_A100", "locations": ["ewr"]},
                {"id": "vc2-1c-1gb", "type": "vc2", "vcpu_count": 1, "ram": 1024, "disk": 25, "monthly_cost": 5,
                 "locations": ["ewr"]}], "meta": {"links": {"next": ""}}})
        if p == "/v2/plans-metal":
            return httpx.Response(200, json={"plans_metal": [
                {"id": "vbm-256c-2048gb-8-mi355x-gpu", "cpu_count": 128, "cpu_threads": 256, "ram": 3145728,
                 "disk": 3840, "disk_count": 4, "monthly_cost": 15768, "hourly_cost": 21.6,
                 "locations": ["ewr", "atl"]}], "meta": {"links": {"next": ""}}})
        if p.startswith("/v2/regions/") and p.endswith("/availability"):
            region = p.split("/")[3]
            plans = {"ewr": ["vbm-256c-2048gb-8-mi355x-gpu", "vcg-a100-12c-120g-80vram"], "atl": []}[region]
            return httpx.Response(200, json={"available_plans": plans})
        return httpx.Response(404)

    c = compute_class(BackendType.VULTR)({}, {"api_key": "k"}, _client(handler))
    mi = {o.region: o for o in c.get_offers(_req(gpu="MI355X:8"))}
    assert mi["ewr"].availability == IA.AVAILABLE and mi["atl"].availability == IA.NOT_AVAILABLE
    assert mi["ewr"].price == 21.6 and mi["ewr"].instance.resources.cpus == 256
    assert mi["ewr"].instance.resources.disk.size_mib == 4 * 3840 * 1024
    a100 = c.get_offers(_req(gpu="A100"))
    assert [o.instance.name for o in a100] == ["vcg-a100-12c-120g-80vram"]  # the 4 GB slice is dropped
    assert a100[0].price == round(1750 / 730, 4)


def test_datacrunch_live_listing(live):
    def handler(req):
        p = req.url.path
        if p.endswith("/oauth2/token"):
            return httpx.Response(200, json={"access_token": "t", "expires_in": 3600})
        if p.endswith("/instance-types"):
            return httpx.Response(200, json=[{
                "instance_type": "8H100.80S.176V", "price_per_hour": "21.92", "spot_price": "7.5",
                "cpu": {"number_of_cores": 176}, "memory": {"size_in_gigabytes": 1480},
                "gpu": {"number_of_gpus": 8, "description": "8x H100 SXM5 80GB"},
                "gpu_memory": {"size_in_gigabytes": 640}}])
        if p.endswith("/instance-availability"):
            spot = req.url.params["is_spot"] == "true"
            return httpx.Response(200, json=[
                {"location_code": "FIN-01", "availabilities": [] if spot else ["8H100.80S.176V"]},
                {"location_code": "ICE-01", "availabilities": ["8H100.80S.176V"] if spot else []}])
        return httpx.Response(404)

    c = compute_class(BackendType.DATACRUNCH)({}, {"client_id": "a", "client_secret": "b"}, _client(handler))
    offers = {(o.region, o.instance.resources.spot): o for o in c.get_offers(_req(gpu="H100:8"))}
    assert offers[("FIN-01", False)].availability == IA.AVAILABLE
    assert offers[("FIN-01", True)].availability == IA.NOT_AVAILABLE
    assert offers[("ICE-01", True)].availability == IA.AVAILABLE and offers[("ICE-01", True)].price == 7.5
    assert offers[("FIN-01", False)].instance.resources.gpus[0].memory_mib == 80 * 1024


def test_tensordock_live_listing_and_launch(live):
    launched = {}

    def handler(req):
        p = req.url.path
        if p.endswith("/client/deploy/hostnodes"):
            return httpx.Response(200, json={"success": True, "hostnodes": {"node-1": {
                "location": {"country": "United States", "region": "Texas", "city": "Dallas"},
                "status": {"online": True},
                "specs": {"cpu": {"amount": 64, "price": 0.003}, "ram": {"amount": 512, "price": 0.002},
                          "storage": {"amount": 4000, "price": 0.0001},
                          "gpu": {"mi300x-oam-192gb": {"amount": 4, "price": 2.0, "vram": 192}}}}}})
        if p.endswith("/client/deploy/single"):
            launched.update(dict(urllib.parse.parse_qsl(req.content.decode())))
            return httpx.Response(200, json={"success": True, "server": "vm-1", "ip": "1.2.3.4",
                                             "port_forwards": {"20022": "22"}})
        return httpx.Response(404)

    c = compute_class(BackendType.TENSORDOCK)({}, {"api_key": "k", "api_token": "t"}, _client(handler))
    offers = c.get_offers(_req(gpu="MI300X:1.."))
    assert sorted(len(o.instance.resources.gpus) for o in offers) == [1, 2, 4]
    two = next(o for o in offers if len(o.instance.resources.gpus) == 2)
    assert two.instance.name == "mi300x-oam-192gb:2:node-1" and two.region == "unitedstates-texas-dallas"
    assert two.instance.resources.cpus == 32 and two.instance.resources.memory_mib == 256 * 1024
    assert two.price == pytest.approx(2 * 2.0 + 32 * 0.003 + 256 * 0.002 + 100 * 0.0001)
    from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey

    cfg = InstanceConfiguration(project_name="main", instance_name="r-0", user="admin",
                                ssh_keys=[SSHKey(public="ssh-ed25519 AAAA k")])
    jpd = c.create_instance(two, cfg)
    assert launched["hostnode"] == "node-1" and launched["gpu_model"] == "mi300x-oam-192gb"
    assert launched["gpu_count"] == "2" and jpd.ssh_port == 20022
    script = launched["cloudinit_script"]  # one line, newlines escaped, as the form field expects
    assert "\n" not in script and script.startswith("#cloud-config\\n") and "dstack-shim" in script


def test_runpod_live_listing_feeds_run_job(live):
    sent = []

    def handler(req):
        body = json.loads(req.content)
        sent.append(body)
        if "gpuTypes" in body["query"]:
            return httpx.Response(200, json={"data": {
                "gpuTypes": [{"id": "AMD Instinct MI300X OAM", "displayName": "MI300X", "memoryInGb": 192,
                              "maxGpuCount": 8, "securePrice": 2.49, "secureSpotPrice": 1.99,
                              "lowestPrice": {"minVcpu": 24, "minMemory": 283}}],
                "dataCenters": [
                    {"id": "EU-RO-1", "listed": True,
                     "gpuAvailability": [{"gpuTypeId": "AMD Instinct MI300X OAM", "available": True,
                                          "stockStatus": "High"}]},
                    {"id": "US-TX-3", "listed": True,
                     "gpuAvailability": [{"gpuTypeId": "AMD Instinct MI300X OAM", "available": False,
                                          "stockStatus": None}]}]}})
        return httpx.Response(200, json={"data": {"podFindAndDeployOnDemand": {"id": "pod-1", "machineId": "m"}}})

    c = compute_class(BackendType.RUNPOD)({}, {"api_key": "k"}, _client(handler))
    offers = c.get_offers(_req(gpu="MI300X:8", spot=False))
    by = {o.region: o for o in offers}
    assert by["EU-RO-1"].availability == IA.AVAILABLE and by["US-TX-3"].availability == IA.NOT_AVAILABLE
    assert by["EU-RO-1"].price == pytest.approx(8 * 2.49) and by["EU-RO-1"].instance.resources.cpus == 192
    from types import SimpleNamespace

    run = SimpleNamespace(run_spec=SimpleNamespace(run_name="r", ssh_key_pub=""))
    job = SimpleNamespace(job_spec=SimpleNamespace(job_num=0, image_name=None))
    c.run_job(run, job, by["EU-RO-1"], "ssh-ed25519 K", "", [])
    assert sent[-1]["variables"]["input"]["gpuTypeId"] == "AMD Instinct MI300X OAM"
    assert sent[-1]["variables"]["input"]["gpuCount"] == 8


def test_vastai_live_listing(live):
    def handler(req):
        assert req.url.path == "/api/v0/bundles/"
        return httpx.Response(200, json={"offers": [
            {"id": 77, "gpu_name": "RTX 4090", "num_gpus": 2, "gpu_ram": 24564, "cpu_cores_effective": 16,
             "cpu_ram": 65536, "disk_space": 200, "dph_total": 0.8, "geolocation": "US"}]})

    c = compute_class(BackendType.VASTAI)({}, {"api_key": "k"}, _client(handler))
    (o,) = c.get_offers(None)
    assert o.instance.name == "77" and o.price == 0.8 and o.availability == IA.AVAILABLE
    assert o.instance.resources.memory_mib == 64 * 1024 and len(o.instance.resources.gpus) == 2


def _ec2(body):
    return httpx.Response(200, text=f'<R xmlns="http://ec2.amazonaws.com/doc/2016-11-15/">{body}</R>')


def test_aws_live_overlay_offerings_spot_and_quota(live):
    def handler(req):
        host = req.url.host
        if host.startswith("servicequotas."):
            region = host.split(".")[1]
            assert req.headers["x-amz-target"] == "ServiceQuotasV20190624.ListServiceQuotas"
            p_quota = 0 if region == "us-west-2" else 384
            return httpx.Response(200, json={"Quotas": [
                {"QuotaName": "Running On-Demand P instances", "Value": p_quota,
                 "UsageMetric": {"MetricDimensions": {"Class": "P/OnDemand"}}},
                {"QuotaName": "All P Spot Instance Requests", "Value": 192,
                 "UsageMetric": {"MetricDimensions": {"Class": "P/Spot"}}}]})
        region = host.split(".")[1]
        form = dict(urllib.parse.parse_qsl(req.content.decode()))
        if form["Action"] == "DescribeInstanceTypeOfferings":
            offered = {"us-east-1": ["p5.48xlarge", "g5.xlarge", "c6i.xlarge"], "us-west-2": ["p5.48xlarge"],
                       "eu-west-1": []}[region]
            return _ec2("<instanceTypeOfferingSet>" + "".join(
                f"<item><instanceType>{t}</instanceType></item>" for t in offered) + "</instanceTypeOfferingSet>")
        if form["Action"] == "DescribeSpotPriceHistory":
            assert form["ProductDescription.1"] == "Linux/UNIX"
            return _ec2("<spotPriceHistorySet>"
                        "<item><instanceType>p5.48xlarge</instanceType><spotPrice>31.5</spotPrice></item>"
                        "<item><instanceType>p5.48xlarge</instanceType><spotPrice>29.25</spotPrice></item>"
                        "</spotPriceHistorySet>")
        return httpx.Response(400, text="<Response><Errors><Error><Code>X</Code></Error></Errors></Response>")

    c = compute_class(BackendType.AWS)({}, {"access_key": "AK", "secret_key": "SK"}, _client(handler))
    p5 = {(o.region, o.instance.resources.spot): o for o in c.get_offers(_req(gpu="H100:8"))}
    assert p5[("us-east-1", False)].availability == IA.UNKNOWN
    assert p5[("us-west-2", False)].availability == IA.NO_QUOTA  # P/OnDemand quota 0 vCPUs
    assert p5[("us-east-1", True)].price == 29.25 and p5[("us-east-1", True)].availability == IA.UNKNOWN
    g5 = {o.region: o.availability for o in c.get_offers(_req(gpu="A10G"))}
    assert g5 == {"us-east-1": IA.UNKNOWN, "eu-west-1": IA.NOT_AVAILABLE}


def test_aws_quota_classes():
    from dstack_amd.core.backends.clouds.aws import quota_class

    assert quota_class("p5.48xlarge", False) == "P/OnDemand"
    assert quota_class("g6e.xlarge", True) == "G/Spot"
    assert quota_class("trn1.32xlarge", False) == "Trn/OnDemand"
    assert quota_class("inf2.xlarge", False) == "Inf/OnDemand"
    assert quota_class("c6i.xlarge", False) == "Standard/OnDemand"


def test_azure_live_retail_prices_and_restrictions(live):
    def handler(req):
        if req.url.host == "prices.azure.com":
            flt = req.url.params.get("$filter", "")
            if "armSkuName eq 'Standard_ND96isr_MI300X_v5'" not in flt:
                return httpx.Response(400)
            if req.url.params.get("page") == "2":
                return httpx.Response(200, json={"Items": [
                    {"armSkuName": "Standard_ND96isr_MI300X_v5", "armRegionName": "westus", "retailPrice": 47.0,
                     "skuName": "ND96isr MI300X v5", "productName": "NDisrMI300Xv5 Series", "unitOfMeasure": "1 Hour"}],
                    "NextPageLink": None})
            return httpx.Response(200, json={"Items": [
                {"armSkuName": "Standard_ND96isr_MI300X_v5", "armRegionName": "eastus", "retailPrice": 45.5,
                 "skuName": "ND96isr MI300X v5", "productName": "NDisrMI300Xv5 Series", "unitOfMeasure": "1 Hour"},
                {"armSkuName": "Standard_ND96isr_MI300X_v5", "armRegionName": "eastus", "retailPrice": 9.1,
                 "skuName": "ND96isr MI300X v5 Spot", "productName": "NDisrMI300Xv5 Series", "unitOfMeasure": "1 Hour"},
                {"armSkuName": "Standard_ND96isr_MI300X_v5", "armRegionName": "eastus", "retailPrice": 60.0,
                 "skuName": "ND96isr MI300X v5", "productName": "NDisrMI300Xv5 Series Windows",
                 "unitOfMeasure": "1 Hour"},
                {"armSkuName": "Standard_ND96isr_MI300X_v5", "armRegionName": "swedencentral", "retailPrice": 50.0,
                 "skuName": "ND96isr MI300X v5", "productName": "NDisrMI300Xv5 Series", "unitOfMeasure": "1 Hour"}],
                "NextPageLink": "https://prices.azure.com/api/retail/prices?" + urllib.parse.urlencode(
                    {"$filter": flt, "page": "2"})})
        if req.url.host == "login.microsoftonline.com":
            return httpx.Response(200, json={"access_token": "t", "expires_in": 3600})
        if req.url.path.endswith("/providers/Microsoft.Compute/skus"):
            return httpx.Response(200, json={"value": [{
                "resourceType": "virtualMachines", "name": "Standard_ND96isr_MI300X_v5",
                "restrictions": [{"type": "Location", "reasonCode": "NotAvailableForSubscription",
                                  "values": ["swedencentral"],
                                  "restrictionInfo": {"locations": ["swedencentral"]}}]}]})
        return httpx.Response(404)

    c = compute_class(BackendType.AZURE)({"subscription_id": "sub", "tenant_id": "ten"},
                                         {"client_id": "c", "client_secret": "s"}, _client(handler))
    offers = {(o.region, o.instance.resources.spot): o for o in c.get_offers(_req(gpu="MI300X:8"))}
    assert set(offers) == {("eastus", False), ("eastus", True), ("westus", False), ("swedencentral", False)}
    assert offers[("eastus", False)].price == 45.5 and offers[("eastus", True)].price == 9.1
    assert offers[("westus", False)].price == 47.0
    assert offers[("swedencentral", False)].availability == IA.NO_QUOTA
    assert offers[("eastus", False)].instance.resources.cpus == 96


def test_azure_locations_filter_offers():
    """Azure configs name their regions ``locations``; they filter the offers like ``regions``."""
    c = compute_class(BackendType.AZURE)({"locations": ["westus"], "subscription_id": "s", "tenant_id": "t"}, {})
    assert {o.region for o in c.get_offers(_req(gpu="MI300X:8"))} == {"westus"}


def test_gcp_live_machine_types_and_launch_zone(live, monkeypatch):
    from dstack_amd.core.backends.clouds import hyperscalers

    monkeypatch.setattr(hyperscalers.GCPCompute, "_h", lambda self: {"Authorization": "Bearer t"})
    inserted = []

    def handler(req):
        if req.url.path.endswith("/aggregated/machineTypes"):
            assert 'name = "a3-highgpu-8g"' in req.url.params["filter"]
            return httpx.Response(200, json={"items": {
                "zones/us-central1-c": {"machineTypes": [{"name": "a3-highgpu-8g"}, {"name": "e2-standard-4"}]},
                "zones/europe-west4-b": {"machineTypes": [{"name": "a3-highgpu-8g"}]},
                "zones/asia-east1-a": {"warning": {"code": "NO_RESULTS_ON_PAGE"}}}})
        if req.method == "POST" and req.url.path.endswith("/instances"):
            inserted.append(req.url.path)
            return httpx.Response(200, json={"name": "op"})
        return httpx.Response(404)

    c = compute_class(BackendType.GCP)({"project_id": "p"}, {"data": json.dumps({"client_email": "x"})},
                                       _client(handler))
    offers = {(o.region, o.instance.resources.spot): o for o in c.get_offers(_req(gpu="H100:8"))}
    assert set(offers) == {("us-central1", False), ("us-central1", True), ("europe-west4", False),
                           ("europe-west4", True)}
    assert all(o.availability == IA.UNKNOWN for o in offers.values())
    from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey

    cfg = InstanceConfiguration(project_name="main", instance_name="r-0", user="admin",
                                ssh_keys=[SSHKey(public="ssh-ed25519 AAAA k")])
    c.create_instance(offers[("europe-west4", False)], cfg)
    assert "/zones/europe-west4-b/instances" in inserted[0]


def test_oci_live_shapes_per_availability_domain(live, monkeypatch):
    from dstack_amd.core.backends.clouds import hyperscalers

    monkeypatch.setattr(hyperscalers, "rsa_sha256_sign", lambda key, data: b"sig")

    def handler(req):
        region = req.url.host.split(".")[1]
        if req.url.path.endswith("/availabilityDomains"):
            return httpx.Response(200, json=[{"name": f"Xy:{region.upper()}-AD-1"}, {"name": f"Xy:{region.upper()}-AD-2"}])
        if req.url.path.endswith("/shapes"):
            q = dict(urllib.parse.parse_qsl(req.url.query.decode()))
            has = region == "us-chicago-1" and q["availabilityDomain"].endswith("AD-2")
            if q.get("page") == "p2":
                return httpx.Response(200, json=[{"shape": "BM.GPU.MI355X.8"}] if has else [])
            return httpx.Response(200, json=[{"shape": "VM.Standard.E5.Flex"}], headers={"opc-next-page": "p2"})
        return httpx.Response(404)

    c = compute_class(BackendType.OCI)({"regions": ["us-chicago-1", "eu-frankfurt-1"], "compartment_id": "comp"},
                                       {"tenancy": "ten", "user": "u", "fingerprint": "fp", "key_content": "k"},
                                       _client(handler))
    offers = {o.region: o.availability for o in c.get_offers(_req(gpu="MI355X:8"))}
    assert offers == {"us-chicago-1": IA.UNKNOWN, "eu-frankfurt-1": IA.NOT_AVAILABLE}
    assert c._ad_for("us-chicago-1", "BM.GPU.MI355X.8") == "Xy:US-CHICAGO-1-AD-2"


def test_gcp_launch_finds_zone_without_a_listing(monkeypatch):
    """Offers from the offline catalog (no live listing in this process): the launch still asks
    which zone of the region offers the machine type instead of assuming '<region>-a'."""
    from dstack_amd.core.backends.clouds import hyperscalers
    from dstack_amd.core.models.instances import InstanceConfiguration, SSHKey

    monkeypatch.setattr(hyperscalers.GCPCompute, "_h", lambda self: {"Authorization": "Bearer t"})
    inserted = []

    def handler(req):
        if req.url.path.endswith("/aggregated/machineTypes"):
            return httpx.Response(200, json={"items": {"zones/us-central1-f": {"machineTypes": [
                {"name": "a3-highgpu-8g"}]}}})
        if req.method == "POST":
            inserted.append(req.url.path)
            return httpx.Response(200, json={"name": "op"})
        return httpx.Response(404)

    c = compute_class(BackendType.GCP)({"project_id": "p"}, {"data": json.dumps({"client_email": "x"})},
                                       _client(handler))
    offer = next(o for o in c.get_offers(_req(gpu="H100:8")) if o.region == "us-central1")
    cfg = InstanceConfiguration(project_name="main", instance_name="r-0", user="admin",
                                ssh_keys=[SSHKey(public="ssh-ed25519 AAAA k")])
    c.create_instance(offer, cfg)
    assert "/zones/us-central1-f/instances" in inserted[0]


def test_live_listing_is_cached_per_credentials(live):
    n = {"calls": 0}

    def handler(req):
        n["calls"] += 1
        return httpx.Response(200, json={"data": {}})

    a = compute_class(BackendType.LAMBDA)({}, {"api_key": "a"}, _client(handler))
    a.get_offers(None)
    a._offers_cache.clear()
    a.get_offers(None)
    assert n["calls"] == 1  # the online cache answered the second query
    b = compute_class(BackendType.LAMBDA)({}, {"api_key": "b"}, _client(handler))
    b.get_offers(None)
    assert n["calls"] == 2  # another account -> its own listing
    assert a.catalog_key() != b.catalog_key()


def test_catalog_rows_report_layer(live):
    rows, layer = catalog.catalog_rows(BackendType.VULTR)
    assert layer == "offline" and rows
    rows, layer = catalog.catalog_rows(BackendType.VULTR, lambda: [gpu_row("x", "y", 1, 1, 1, None, 0)], "k")
    assert layer == "online" and rows[0].instance_name == "x"
    assert get_catalog_offers(BackendType.VULTR, rows=rows)[0].instance.name == "x"
