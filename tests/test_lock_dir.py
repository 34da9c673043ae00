"""Where the per-GPU launch lock lives (fit_lock_dir).

The lock serialises the persistent launches of every engine on one GPU, across processes.  The
configurator runs each virtual kubelet as its own pod (reference pkg/configurator/configurator.go:
188-293), whose /tmp is private, so the default is the /var/run/fitgpu host path that the VK pod
template mounts; /tmp is only a fallback, reported as not shared.  CPU
only: resolving the directory needs no device."""
import ctypes as C
import os

from fitgpu import _lib
import fitgpu

DEFAULT = "/var/run/fitgpu"


def test_override_is_used(monkeypatch, tmp_path):
    monkeypatch.setenv("FIT_LOCK_DIR", str(tmp_path))
    assert fitgpu.lock_dir() == (str(tmp_path), True)


def test_default_host_path_or_reported_fallback(monkeypatch):
    monkeypatch.delenv("FIT_LOCK_DIR", raising=False)
    d, shared = fitgpu.lock_dir()
    if os.path.isdir(DEFAULT):
        assert (d, shared) == (DEFAULT, True)
    else:
        assert (d, shared) == ("/tmp", False)


def test_empty_override_means_unset(monkeypatch):
    monkeypatch.setenv("FIT_LOCK_DIR", "")
    d, _ = fitgpu.lock_dir()
    assert d in (DEFAULT, "/tmp")


def test_small_buffer_is_rejected(monkeypatch, tmp_path):
    monkeypatch.setenv("FIT_LOCK_DIR", str(tmp_path))
    buf = C.create_string_buffer(4)
    assert _lib.lib().fit_lock_dir(buf, len(buf)) == _lib.FIT_E_INVAL
