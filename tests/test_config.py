"""CLI contract: the reference's 11 flags, defaults, types and help (reference train_ddp.py:19-46)."""
import pytest

from distributed_pytorch_training_amd.config import build_parser, parse_args

REFERENCE_FLAGS = {
    "data_dir": ("./data", "directory to store CIFAR-10"),
    "epochs": (10, "number of total epochs to run"),
    "batch_size": (128, "mini-batch size *per GPU*"),
    "workers": (4, "number of data loading workers per process"),
    "lr": (0.1, "initial learning rate"),
    "momentum": (0.9, "SGD momentum"),
    "weight_decay": (5e-4, "weight decay"),
    "amp": (False, "use automatic mixed precision (AMP)"),
    "print_freq": (50, "print frequency (in steps)"),
    "output_dir": ("./experiments", "directory to save logs"),
    "seed": (42, "random seed"),
}


def test_reference_defaults_and_help():
    p = build_parser()
    assert p.description == "DDP training of ResNet-18 on CIFAR-10"
    acts = {a.dest: a for a in p._actions}
    for dest, (default, help_) in REFERENCE_FLAGS.items():
        assert acts[dest].default == default, dest
        assert acts[dest].help == help_, dest
    args = parse_args([])
    for dest, (default, _) in REFERENCE_FLAGS.items():
        assert getattr(args, dest) == default


def test_additive_defaults_reproduce_reference():
    a = parse_args([])
    assert a.model == "resnet18" and a.dataset == "cifar10"
    assert a.image_size == 32 and a.num_classes == 10
    assert a.amp_dtype == "fp16" and a.optimizer == "sgd"
    assert a.bucket_cap_mb == 25.0 and a.first_bucket_mb == 1.0
    assert a.broadcast_buffers is True and a.grad_dtype == "fp32"
    assert a.save_every == 0 and a.resume is None


def test_types_and_overrides():
    a = parse_args(["--epochs", "3", "--batch-size", "64", "--lr", "0.05", "--amp",
                    "--dataset", "synthetic", "--backend", "nccl", "--betas", "0.8,0.9"])
    assert a.epochs == 3 and a.batch_size == 64 and a.lr == 0.05 and a.amp
    assert a.image_size == 224 and a.num_classes == 1000  # synthetic = ImageNet shape
    assert a.backend == "rccl" and a.betas == (0.8, 0.9)
    with pytest.raises(SystemExit):
        parse_args(["--epochs", "x"])


def test_rehearse_shared_gpu_needs_a_host_bridge(monkeypatch, tmp_path):
    """--rehearse-shared-gpu (testing: N ranks on one GPU) is off by default and refuses a
    communicator that needs one GPU per rank before touching the process group."""
    from distributed_pytorch_training_amd.engine import run
    assert parse_args([]).rehearse_shared_gpu is False
    for k, v in {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}.items():
        monkeypatch.setenv(k, v)
    with pytest.raises(SystemExit, match="host-async"):
        run.main(["--dataset", "synthetic", "--rehearse-shared-gpu", "--comm", "rccl",
                  "--output-dir", str(tmp_path)])


def test_shared_gpu_bootstrap_needs_a_gpu(monkeypatch):
    from distributed_pytorch_training_amd.utils import dist as udist
    for k, v in {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(udist, "gpu_available", lambda: False)
    with pytest.raises(RuntimeError, match="visible GPU"):
        udist.init_distributed("auto", 30, shared_gpu=True)
