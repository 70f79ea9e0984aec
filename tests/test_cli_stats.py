"""``dstack stats`` renders per-GPU amdsmi figures: memory, util, power, HBM activity, xGMI
throughput and links (fake client; the metric names are the server's, services/metrics.py)."""

from types import SimpleNamespace

from dstack_amd.cli import commands


def test_stats_shows_gpu_power_hbm_and_xgmi(monkeypatch, capsys):
    def metric(name, v):
        return SimpleNamespace(name=name, values=[v])

    metrics = SimpleNamespace(metrics=[
        metric("cpu_usage_percent", 250.0), metric("memory_working_set_bytes", 8 << 30),
        metric("gpus_detected_num", 1.0), metric("gpu_util_percent_gpu0", 97.0),
        metric("gpu_memory_usage_bytes_gpu0", float(171 << 30)), metric("gpu_power_watts_gpu0", 1330.0),
        metric("gpu_hbm_activity_percent_gpu0", 64.0), metric("gpu_xgmi_read_bytes_per_s_gpu0", 2.5e11),
        metric("gpu_xgmi_write_bytes_per_s_gpu0", 2.4e11), metric("gpu_xgmi_links_up_gpu0", 7.0),
    ])
    job = SimpleNamespace(job_spec=SimpleNamespace(job_name="train-0-0", replica_num=0, job_num=0))
    run = SimpleNamespace(refresh=lambda: SimpleNamespace(model=SimpleNamespace(jobs=[job])))
    client = SimpleNamespace(project="main", runs=SimpleNamespace(get=lambda name: run),
                             api=SimpleNamespace(metrics=SimpleNamespace(get_job_metrics=lambda *a: metrics)))
    monkeypatch.setattr(commands, "_client", lambda args: client)
    monkeypatch.setattr(commands, "print_table", lambda t: commands.console.print(t, width=200))
    assert commands.cmd_stats(SimpleNamespace(run_name="train", watch=False, project=None)) == 0
    out = " ".join(capsys.readouterr().out.split())  # the table may wrap the GPU column
    assert "97.0% util" in out and "1330W" in out and "HBM 64%" in out
    assert "xGMI rd 250.0 wr 240.0 GB/s" in out and "(7 links up)" in out
