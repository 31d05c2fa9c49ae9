"""TensorBoard scalar event files written without tensorboard (the
reference trainer's SummaryWriter(args.dir): 'loss' per log interval,
'accuracy' per epoch, examples/mnist/mnist.py:49,65,108)."""
import glob
import os
import struct

from pytorch_operator_1_amd.utils import tbevents


def test_crc32c_known_vector():
    assert tbevents.crc32c(b"123456789") == 0xE3069283


def test_writer_roundtrip(tmp_path):
    with tbevents.SummaryWriter(str(tmp_path)) as w:
        for i in range(5):
            w.add_scalar("loss", 1.0 / (i + 1), i * 10)
        w.add_scalar("accuracy", 0.9664, 1)
    (path,) = glob.glob(os.path.join(tmp_path, "events.out.tfevents.*"))
    rows = tbevents.read_scalars(path)
    assert [(s, t) for s, t, _ in rows] == [(0, "loss"), (10, "loss"), (20, "loss"), (30, "loss"), (40, "loss"),
                                            (1, "accuracy")]
    assert abs(rows[-1][2] - 0.9664) < 1e-6
    # TFRecord framing: first record is the file_version event
    data = open(path, "rb").read()
    (n,) = struct.unpack_from("<Q", data, 0)
    assert b"brain.Event:2" in data[12:12 + n]


def test_trainer_writes_loss_and_accuracy(tmp_path, monkeypatch):
    from pytorch_operator_1_amd.train import mnist

    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    d = tmp_path / "tb"
    rc = mnist.main(["--no-cuda", "--max-steps", "12", "--log-interval", "5", "--train-size", "640",
                     "--test-size", "128", "--dir", str(d)])
    assert rc == 0
    (path,) = glob.glob(os.path.join(d, "events.out.tfevents.*"))
    rows = tbevents.read_scalars(path)
    tags = [t for _, t, _ in rows]
    assert tags.count("loss") >= 2 and tags.count("accuracy") == 1
