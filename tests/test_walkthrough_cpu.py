"""The reference notebook's end-to-end flow on one box (examples/walkthrough_cifar10_tensorboard.py): a
CIFAR-10-shaped ResNet TfJob with a TensorBoard section, polled to Done, its loss curve read back through the
TensorBoard Service's HTTP API; plus the TensorBoard stand-in over hand-written event files."""
import importlib.util
import json
import os
import socket
import threading
import urllib.request

from k8s_amd.tools import tensorboard as tbmod
from k8s_amd.utils.tfevents import EventWriter, read_events

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load_walkthrough():
    spec = importlib.util.spec_from_file_location("walkthrough",
                                                  os.path.join(REPO, "examples", "walkthrough_cifar10_tensorboard.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_walkthrough_job_to_done_with_tensorboard(tmp_path):
    out = _load_walkthrough().run(steps=12, logdir=str(tmp_path / "logs"), timeout=300, verbose=False)
    assert out["phase"] == "Done" and out["state"] == "Succeeded"
    assert "loss" in out["tags"]["."] and "learning_rate" in out["tags"]["."]
    assert out["loss_points"] >= 2 and out["loss_steps"] == sorted(out["loss_steps"])
    assert out["loss_steps"][-1] == 11


def test_tensorboard_standin_serves_scalars(tmp_path):
    w = EventWriter(str(tmp_path / "run1"))
    for step in range(5):
        w.scalars(step, {"loss": 1.0 / (step + 1), "acc": step * 0.1})
    w.flush()
    evs = list(read_events(w.path))
    assert evs[0].get("file_version") == "brain.Event:2" and abs(evs[3]["scalars"]["loss"] - 1.0 / 3) < 1e-6
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    from http.server import ThreadingHTTPServer

    srv = ThreadingHTTPServer(("127.0.0.1", port), tbmod.make_handler(tbmod.EventStore(str(tmp_path))))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        base = "http://127.0.0.1:%d" % port
        get = lambda p: json.loads(urllib.request.urlopen(base + p, timeout=5).read())  # noqa: E731
        assert get("/data/runs") == ["run1"]
        assert set(get("/data/plugin/scalars/tags")["run1"]) == {"loss", "acc"}
        series = get("/data/plugin/scalars/scalars?run=run1&tag=loss")
        assert [p[1] for p in series] == [0, 1, 2, 3, 4] and abs(series[4][2] - 0.2) < 1e-6
        w.scalars(5, {"loss": 0.1})  # appended after the first scan: picked up incrementally
        w.flush()
        assert len(get("/data/plugin/scalars/scalars?run=run1&tag=loss")) == 6
    finally:
        srv.shutdown()
        w.close()
