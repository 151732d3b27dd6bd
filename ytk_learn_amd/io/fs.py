"""File-system abstraction (reference: ``J/fs/IFileSystem.java``, ``LocalFileSystem.java``,
``HdfsFileSystem.java``, ``FileSystemFactory.java:54-63``).

``fs_scheme`` values: ``local`` / ``file:///`` -> :class:`LocalFileSystem`; any other
scheme (``hdfs://``, ``s3://`` ...) goes through ``fsspec`` when a driver for it is
importable, otherwise a clear error. Hidden files (``.name`` / ``_name``) are skipped
by recursive listing, as in the reference.
"""
from __future__ import annotations

import io
import os
import shutil
from typing import IO, Iterable, Iterator, List, Sequence

from ..utils.errors import YtkLearnError


def _hidden(name: str) -> bool:
    return name.startswith(".") or name.startswith("_")


class FileSystem:
    scheme = "base"

    def exists(self, path: str) -> bool:
        raise NotImplementedError

    def open_read(self, path: str, binary: bool = False) -> IO:
        raise NotImplementedError

    def open_write(self, path: str, binary: bool = False, append: bool = False) -> IO:
        raise NotImplementedError

    def is_dir(self, path: str) -> bool:
        raise NotImplementedError

    def list_dir(self, path: str) -> List[str]:
        raise NotImplementedError

    def delete(self, path: str):
        raise NotImplementedError

    def mkdirs(self, path: str):
        raise NotImplementedError

    def local_path(self, path: str):
        """Path usable by native readers, or None when the FS is remote."""
        return None

    # shared helpers -----------------------------------------------------------
    def recur_get_paths(self, paths: Sequence[str]) -> List[str]:
        """All non-hidden regular files under ``paths`` (files or directories), sorted per dir."""
        out: List[str] = []
        for p in paths:
            if not p:
                continue
            if not self.exists(p):
                raise YtkLearnError(f"path not exist: {p}")
            if self.is_dir(p):
                for name in sorted(self.list_dir(p)):
                    if _hidden(name):
                        continue
                    out.extend(self.recur_get_paths([os.path.join(p, name)]))
            else:
                out.append(p)
        return out

    def read_lines(self, path: str) -> Iterator[str]:
        with self.open_read(path) as f:
            for line in f:
                yield line.rstrip("\n").rstrip("\r")

    def read_bytes(self, path: str) -> bytes:
        with self.open_read(path, binary=True) as f:
            return f.read()


class LocalFileSystem(FileSystem):
    scheme = "local"

    @staticmethod
    def _p(path: str) -> str:
        if path.startswith("file://"):
            path = path[len("file://"):]
        return path

    def exists(self, path):
        return os.path.exists(self._p(path))

    def open_read(self, path, binary=False):
        return open(self._p(path), "rb" if binary else "r", encoding=None if binary else "utf-8")

    def open_write(self, path, binary=False, append=False):
        p = self._p(path)
        d = os.path.dirname(p)
        if d:
            os.makedirs(d, exist_ok=True)
        if append:
            return open(p, "ab" if binary else "a", encoding=None if binary else "utf-8")
        return _AtomicWriter(p, binary)

    def is_dir(self, path):
        return os.path.isdir(self._p(path))

    def list_dir(self, path):
        return os.listdir(self._p(path))

    def delete(self, path):
        p = self._p(path)
        if os.path.isdir(p):
            shutil.rmtree(p)
        elif os.path.exists(p):
            os.remove(p)

    def mkdirs(self, path):
        os.makedirs(self._p(path), exist_ok=True)

    def local_path(self, path):
        return self._p(path)


class _AtomicWriter:
    """Write to a hidden temp file next to ``path`` and rename it over ``path`` on a clean
    close, so a worker killed mid-dump never leaves a truncated model / checkpoint behind
    (``continue_train`` then resumes from the previous complete dump). Hidden temp names
    are skipped by ``recur_get_paths``."""

    def __init__(self, path: str, binary: bool):
        d, name = os.path.split(path)
        self.path = path
        self.tmp = os.path.join(d, f".{name}.tmp-{os.getpid()}")
        self.f = open(self.tmp, "wb" if binary else "w", encoding=None if binary else "utf-8")

    def __getattr__(self, name):
        return getattr(self.f, name)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is not None:
            self.f.close()
            os.remove(self.tmp)
            return False
        self.close()
        return False

    def close(self):
        if self.f.closed:
            return
        self.f.flush()
        os.fsync(self.f.fileno())
        self.f.close()
        os.replace(self.tmp, self.path)


class FsspecFileSystem(FileSystem):
    """Remote file systems through fsspec (hdfs/s3/... when the driver is installed)."""

    def __init__(self, scheme: str):
        try:
            import fsspec
            self.fs = fsspec.filesystem(scheme.split("://")[0])
        except Exception as e:  # pragma: no cover - depends on optional drivers
            raise YtkLearnError(f"file system scheme {scheme!r} is not available here: {e}")
        self.scheme = scheme

    def exists(self, path):
        return self.fs.exists(path)

    def open_read(self, path, binary=False):
        f = self.fs.open(path, "rb")
        return f if binary else io.TextIOWrapper(f, encoding="utf-8")

    def open_write(self, path, binary=False, append=False):
        f = self.fs.open(path, "ab" if append else "wb")
        return f if binary else io.TextIOWrapper(f, encoding="utf-8")

    def is_dir(self, path):
        return self.fs.isdir(path)

    def list_dir(self, path):
        return [os.path.basename(p.rstrip("/")) for p in self.fs.ls(path, detail=False)]

    def delete(self, path):
        if self.fs.exists(path):
            self.fs.rm(path, recursive=True)

    def mkdirs(self, path):
        self.fs.makedirs(path, exist_ok=True)


def create_fs(scheme: str = "local") -> FileSystem:
    s = (scheme or "local").strip()
    if s in ("local", "file", "file://", "file:///") or s.startswith("file:"):
        return LocalFileSystem()
    return FsspecFileSystem(s)
