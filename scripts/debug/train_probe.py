"""Probe: loss trajectory memorising one batch -- plain autocast vs bf16 shadow, fused vs MIOpen BN."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from gaussiank_sgd_amd.compression import compressors  # noqa: E402
from gaussiank_sgd_amd.models import resnet50  # noqa: E402
from gaussiank_sgd_amd.parallel import DistributedOptimizer, install_bf16_shadow  # noqa: E402

cuda = torch.device("cuda", 0)
for fused in (True, False):
    for shadow in (False, True):
        for lr in (0.01, 0.001):
            torch.manual_seed(0)
            net = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
            for m in net.modules():
                if hasattr(m, "fused"):
                    m.fused = fused
            base = torch.optim.SGD(net.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
            opt = DistributedOptimizer(base, named_parameters=net.named_parameters(), compression=compressors["none"],
                                       compress_single_rank=True, density_warmup=False)
            if shadow:
                install_bf16_shadow(net, opt)
            g = torch.Generator(device=cuda).manual_seed(1)
            x = torch.randn(32, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
            y = torch.randint(0, 10, (32,), device=cuda, generator=g)
            losses = []
            for _ in range(10):
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = torch.nn.functional.cross_entropy(net(x), y)
                loss.backward()
                opt.step()
                losses.append(round(float(loss), 3))
            print("fused=%s shadow=%s lr=%g: %s" % (fused, shadow, lr, losses), flush=True)
