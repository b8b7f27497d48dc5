"""Build / version information (reference ``VersionInfo``, ``utils/.../version/VersionInfo.scala``:
version, git branch / commit, build time read from a generated properties resource). Here the
values come from the package version and, when available, the repository's git metadata."""
from __future__ import annotations

import os
import subprocess
from dataclasses import asdict, dataclass
from typing import Optional

VERSION = "0.1.0"


@dataclass
class VersionInfo:
    version: str = VERSION
    git_repo_url: Optional[str] = None
    git_branch: Optional[str] = None
    git_commit_id: Optional[str] = None
    build_time: Optional[str] = None

    def to_dict(self):
        return asdict(self)


def _git(*args) -> Optional[str]:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        out = subprocess.run(["git", "-C", root, *args], capture_output=True, text=True, timeout=5)
        return out.stdout.strip() or None if out.returncode == 0 else None
    except (OSError, subprocess.SubprocessError):
        return None


_CACHED: Optional[VersionInfo] = None


def version_info() -> VersionInfo:
    global _CACHED
    if _CACHED is None:
        _CACHED = VersionInfo(git_branch=_git("rev-parse", "--abbrev-ref", "HEAD"),
                              git_commit_id=_git("rev-parse", "HEAD"),
                              git_repo_url=_git("config", "--get", "remote.origin.url"))
    return _CACHED
