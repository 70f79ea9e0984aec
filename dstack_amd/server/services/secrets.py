"""Project secrets (reference: ``S/routers/secrets.py``); values are AES-GCM encrypted at rest."""

from __future__ import annotations

import uuid
from typing import Dict, List

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ResourceNotExistsError
from dstack_amd.core.models.users import Secret
from dstack_amd.server.models import ProjectModel, SecretModel


def list_secrets(s: Session, project: ProjectModel) -> List[Secret]:
    rows = s.execute(select(SecretModel).where(SecretModel.project_id == project.id).order_by(SecretModel.name))
    return [Secret(name=r.name) for r in rows.scalars()]


def get_secret(s: Session, project: ProjectModel, name: str) -> Secret:
    r = s.execute(select(SecretModel).where(SecretModel.project_id == project.id,
                                            SecretModel.name == name)).scalar_one_or_none()
    if r is None:
        raise ResourceNotExistsError(f"Secret {name} not found")
    return Secret(name=r.name, value=r.value)


def add_secret(s: Session, project: ProjectModel, name: str, value: str) -> Secret:
    r = s.execute(select(SecretModel).where(SecretModel.project_id == project.id,
                                            SecretModel.name == name)).scalar_one_or_none()
    if r is None:
        s.add(SecretModel(id=uuid.uuid4(), project_id=project.id, name=name, value=value))
    else:
        r.value = value
    return Secret(name=name)


def delete_secrets(s: Session, project: ProjectModel, names: List[str]):
    for n in names:
        r = s.execute(select(SecretModel).where(SecretModel.project_id == project.id,
                                                SecretModel.name == n)).scalar_one_or_none()
        if r is not None:
            s.delete(r)


def get_project_secrets_mapping(s: Session, project: ProjectModel) -> Dict[str, str]:
    rows = s.execute(select(SecretModel).where(SecretModel.project_id == project.id)).scalars()
    return {r.name: r.value for r in rows}
