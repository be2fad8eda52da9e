"""Child process of tests/test_dist_gpu.py::test_rccl_world1_allgather_and_ddp (run as a fresh
process, so nothing has touched the GPU before the process group is made): a world-size-1 RCCL
("nccl") group on cuda:0 executes the device-side collectives of the config-4 path —
all_gather_packed through all_gather_into_tensor (replay.py) and one DDP learner step — and
checks them against the same work without a process group. Prints one JSON line."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    from blokus_rl_amd import replay
    from blokus_rl_amd.alphazero.learner import DeviceReplay, Learner, alphazero_loss
    from blokus_rl_amd.boards import random_boards
    from blokus_rl_amd.engine import Engine
    from blokus_rl_amd.nets import ResNet

    # deterministic MIOpen backward (no atomic-order rounding): at world size 1 the DDP all-reduce
    # must then leave the gradients bit-identical to the plain backward's
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}

    # (s, pi, z) rows as self-play packs them, gathered over RCCL
    eng = Engine(20, 4, 5)
    states = random_boards(eng, 96, seed0=5, max_plies=40)
    ids, counts = eng.legal_ids(states, cap=1024)
    k = counts.clamp(min=0)
    g = torch.Generator(device="cuda").manual_seed(3)
    pi = torch.rand(ids.shape, device="cuda", generator=g) * (torch.arange(1024, device="cuda") < k.unsqueeze(1))
    z = torch.randint(-1, 4, (96, 4), device="cuda").float()
    buf, cap = replay.pack(states, ids, pi, k, z)
    rows, cap2 = replay.all_gather_packed(buf, cap)
    torch.cuda.synchronize()
    out["allgather_rows"] = int(rows.shape[0])
    out["allgather_equal"] = bool(rows.is_cuda and cap2 == cap and torch.equal(rows, buf))

    # one learner step with DDP over RCCL vs the same step without DDP (same initial weights, batch)
    rb = DeviceReplay(eng, cap=1024)
    rb.add_packed(rows, cap2)
    batch = rb.batch(torch.arange(64, device="cuda") % rows.shape[0])
    torch.manual_seed(0)
    net_a = ResNet(20, 4, eng.A, 1).cuda().train()
    net_b = ResNet(20, 4, eng.A, 1).cuda().train()
    net_b.load_state_dict(net_a.state_dict())
    la = Learner(net_a, batch_size=64)
    out["ddp"] = type(la.net).__name__
    # Learner.train_step's work, split so the gradients can be read before the Adam step
    la.net.train()
    pa, va = la.net(batch["observation"])
    loss_a = alphazero_loss(pa, va, batch, la.policy_fn)
    la.optimizer.zero_grad(set_to_none=True)
    loss_a.backward()
    grads_a = [q.grad.detach().clone() for q in net_a.parameters()]
    la.optimizer.step()
    opt = torch.optim.Adam(net_b.parameters(), lr=1e-3, weight_decay=1e-4)
    p, v = net_b(batch["observation"])
    loss_b = alphazero_loss(p, v, batch)
    opt.zero_grad(set_to_none=True)
    loss_b.backward()
    grads_b = [q.grad.detach().clone() for q in net_b.parameters()]
    opt.step()
    torch.cuda.synchronize()
    out["loss_ddp"], out["loss_plain"] = float(loss_a), float(loss_b)
    # gradients: the DDP all-reduce at world size 1 must leave them as the plain backward's
    out["grad_max_rel_diff"] = max(float((ga - gb).abs().max()) / (float(gb.abs().max()) + 1e-30)
                                   for ga, gb in zip(grads_a, grads_b))
    diff = 0.0
    for (n, pa_), pb in zip(net_a.named_parameters(), net_b.parameters()):
        diff = max(diff, float((pa_.detach() - pb.detach()).abs().max()))
    out["param_max_abs_diff"] = diff
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
