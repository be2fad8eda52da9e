"""Probe MIOpen's fused conv+bias+ReLU / conv+bias+add+ReLU ops (torch.miopen_convolution_relu,
torch.miopen_convolution_add_relu) against conv2d + separate bias/ReLU at the self-play leaf batch
(256 x 64 x 20 x 20, fp32): per-layer time and max deviation, then the whole FusedResNet forward
both ways under graph capture. Run on a GPU box."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from blokus_rl_amd.nets import ResNet, FusedResNet

torch.manual_seed(0)
dev = "cuda"
res = {}


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def graphed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(); fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


for cl in (False, True):
    mf = torch.channels_last if cl else torch.contiguous_format
    x = torch.randn(256, 64, 20, 20, device=dev).contiguous(memory_format=mf)
    z = torch.randn(256, 64, 20, 20, device=dev).contiguous(memory_format=mf)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).contiguous(memory_format=mf)
    b = torch.randn(64, device=dev) * 0.1
    tag = "cl" if cl else "nchw"
    with torch.inference_mode():
        ref = F.relu(F.conv2d(x, w, b, 1, 1))
        ref_add = F.relu(F.conv2d(x, w, b, 1, 1) + z)
        cases = {
            "conv_bias": lambda: F.conv2d(x, w, b, 1, 1),
            "conv_nobias": lambda: F.conv2d(x, w, None, 1, 1),
            "conv_bias_relu": lambda: F.relu(F.conv2d(x, w, b, 1, 1)),
            "miopen_conv_relu": lambda: torch.miopen_convolution_relu(x, w, b, [1, 1], [1, 1], [1, 1], 1),
            "conv_bias_add_relu": lambda: F.relu(F.conv2d(x, w, b, 1, 1) + z),
            "miopen_conv_add_relu": lambda: torch.miopen_convolution_add_relu(x, w, z, 1.0, b, [1, 1], [1, 1], [1, 1], 1),
        }
        for name, fn in cases.items():
            key = f"{tag}_{name}"
            try:
                out = fn()
                ms = timeit(fn)
                r = {"ms": ms}
                if name == "miopen_conv_relu":
                    r["max_abs_dev"] = (out - ref).abs().max().item()
                if name == "miopen_conv_add_relu":
                    r["max_abs_dev"] = (out - ref_add).abs().max().item()
                try:
                    g, _ = graphed(fn)
                    r["graph_ms"] = timeit(g.replay)
                except Exception as ex:  # noqa: BLE001
                    r["graph_error"] = repr(ex)[:200]
            except Exception as ex:  # noqa: BLE001
                r = {"error": repr(ex)[:300]}
            res[key] = r
            print(key, json.dumps(r), flush=True)


# whole network: FusedResNet forward vs a forward on the fused MIOpen ops
class MiopenResNet(torch.nn.Module):
    def __init__(self, f: FusedResNet):
        super().__init__()
        self.f = f

    def forward(self, x):
        f = self.f
        c = lambda conv: (conv.weight, conv.bias)
        w, b = c(f.stem)
        x = torch.miopen_convolution_relu(x, w, b, [1, 1], [1, 1], [1, 1], 1)
        h = x
        n = len(f.blocks)
        for i, (c1, c2) in enumerate(f.blocks):
            h = torch.miopen_convolution_relu(h, c1.weight, c1.bias, [1, 1], [1, 1], [1, 1], 1)
            if i + 1 < n:
                h = F.conv2d(h, c2.weight, c2.bias, 1, 1)
            else:
                h = torch.miopen_convolution_add_relu(h, c2.weight, x, 1.0, c2.bias, [1, 1], [1, 1], [1, 1], 1)
        x = h
        p = torch.miopen_convolution_relu(x, f.policy_conv.weight, f.policy_conv.bias, [1, 1], [0, 0], [1, 1], 1)
        p = F.log_softmax(f.policy_out(p.flatten(1)).float(), dim=1)
        v = torch.miopen_convolution_relu(x, f.value_conv.weight, f.value_conv.bias, [1, 1], [0, 0], [1, 1], 1)
        v = torch.tanh(f.value_fc2(F.relu(f.value_fc1(v.flatten(1))))).float()
        return p, v


net = ResNet(20, 4, 30433, 5).to(dev).eval()
with torch.no_grad():
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.2, 0.2); m.running_var.uniform_(0.5, 1.5)
            m.weight.uniform_(0.8, 1.2); m.bias.uniform_(-0.1, 0.1)
xb = (torch.rand(256, 8, 20, 20, device=dev) < 0.3).float()
with torch.inference_mode():
    ref_p, ref_v = net(xb)
for cl in (False, True):
    fused = FusedResNet(net).eval()
    xx = xb
    if cl:
        fused = fused.to(memory_format=torch.channels_last)
        xx = xb.contiguous(memory_format=torch.channels_last)
    for name, model in (("fused", fused), ("miopen_fused", MiopenResNet(fused))):
        key = f"net_{'cl' if cl else 'nchw'}_{name}"
        try:
            with torch.inference_mode():
                g, (p, v) = graphed(lambda: model(xx))
                ms = timeit(g.replay)
            r = {"graph_ms": ms, "max_abs_dlogp": (p - ref_p).abs().max().item(),
                 "max_abs_dv": (v - ref_v).abs().max().item()}
        except Exception as ex:  # noqa: BLE001
            r = {"error": repr(ex)[:300]}
        res[key] = r
        print(key, json.dumps(r), flush=True)

os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/nn_fused_probe.json", "w"), indent=1)
