"""Airflow DAG that runs dstack-amd jobs on a schedule, two ways:

* ``cli_apply``: the ``dstack`` CLI in a bash task (from a separate virtualenv, so dstack-amd's
  dependencies never clash with Airflow's);
* ``api_train``: the Python API inside a ``@task.external_python`` task in that same virtualenv --
  submit, stream the logs into the Airflow task log, fail the task if the job failed.

Set ``DSTACK_VENV`` to the virtualenv with dstack-amd installed and give the Airflow workers
``DSTACK_SERVER_URL`` / ``DSTACK_TOKEN`` (or a ``~/.dstack/config.yml``).
"""
import os
from datetime import datetime, timedelta

from airflow.configuration import conf
from airflow.decorators import dag, task

REPO_DIR = os.path.join(conf.get("core", "DAGS_FOLDER"), "dstack-repo")
DSTACK_VENV = os.environ.get("DSTACK_VENV", "/opt/dstack-venv")


@dag(schedule=timedelta(days=1), start_date=datetime(2025, 1, 1), catchup=False,
     default_args={"retries": 1, "retry_delay": timedelta(minutes=5)},
     description="Nightly dstack-amd jobs on MI355X")
def dstack_amd_tasks():
    @task.bash
    def cli_apply() -> str:
        return f"source {DSTACK_VENV}/bin/activate && cd {REPO_DIR} && dstack init && dstack apply -y -f task.dstack.yml"

    @task.external_python(python=f"{DSTACK_VENV}/bin/python")
    def api_train(repo_dir: str) -> str:
        import sys

        from dstack_amd.api import GPU, Client, Resources, Task

        client = Client.from_config()
        repo = client.repos.load(repo_dir, init=True)
        run = client.runs.submit(
            Task(name="nightly-eval", commands=["python3 eval.py"],
                 resources=Resources(gpu=GPU(name=["MI355X"], count=1))),
            repo=repo)
        for chunk in run.logs():
            sys.stdout.write(chunk.decode(errors="replace"))
        status = run.wait()
        if status.value != "done":
            raise RuntimeError(f"{run.name} finished as {status.value}")
        return run.name

    cli_apply() >> api_train(REPO_DIR)


dstack_amd_tasks()
