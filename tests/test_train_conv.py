"""CPU side of the learner's device path (alphazero/train_conv.py): the in-place module switch
keeps the reference's parameters and state_dict keys (checkpoints stay interchangeable) and, off
the GPU, computes exactly what nn.Conv2d / nn.BatchNorm2d compute."""
import torch


def test_prepare_model_keeps_state_and_cpu_semantics():
    from blokus_rl_amd.alphazero.train_conv import X3Conv2d, prepare_model, use_x3_convs
    from blokus_rl_amd.nets import NativeBatchNorm2d, ResNet

    torch.manual_seed(0)
    ref = ResNet(20, 4, 100, 2)
    net = ResNet(20, 4, 100, 2)
    net.load_state_dict(ref.state_dict())
    keys = list(net.state_dict())
    prepare_model(net)
    assert list(net.state_dict()) == keys
    assert sum(isinstance(m, X3Conv2d) for m in net.modules()) == 4  # the tower's 64->64 convs only
    assert isinstance(net.conv1, torch.nn.Conv2d) and not isinstance(net.conv1, X3Conv2d)
    assert isinstance(net.bn1, NativeBatchNorm2d)
    assert use_x3_convs(net) == 0  # idempotent
    x = torch.randn(3, 8, 20, 20)
    ref.train()
    net.train()
    p0, v0 = ref(x)
    p1, v1 = net(x.contiguous(memory_format=torch.channels_last))
    assert torch.allclose(p0, p1, atol=1e-5, rtol=1e-5) and torch.allclose(v0, v1, atol=1e-6)
    # the running statistics moved the same way
    assert torch.allclose(ref.bn1.running_mean, net.bn1.running_mean, atol=1e-6)


def test_learner_auto_stays_off_on_cpu():
    from blokus_rl_amd.alphazero.learner import Learner
    from blokus_rl_amd.nets import ResNet

    assert Learner(ResNet(20, 4, 100, 1), batch_size=1024).device_path is False
