"""Debug: per-step loss / NaN state / bucket records of the PTB LSTM on the GPU path."""
import torch

from gaussiank_sgd_amd.compression import compressors
from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
from gaussiank_sgd_amd.train import DLTrainer

torch.manual_seed(0)
comm.init()
t = DLTrainer(0, 1, dnn="lstm", dataset="ptb", batch_size=16, lr=1.0, device="cuda", amp="bf16",
              learnable_data=True, data_pool=1)
opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(), compression=compressors["gaussian"],
                           is_sparse=True, density=0.01, compress_single_rank=True, density_warmup=False)
install_bf16_shadow(t.net, opt)
t.update_optimizer(opt)
hidden = None
for step in range(8):
    opt.zero_grad()
    _, hidden = t.train(1, hidden=hidden)
    opt.synchronize()
    nrm = opt.clip_grad_norm_(0.25)
    torch.cuda.synchronize()
    gn = float(nrm)
    hn = [float(h.float().abs().max()) for h in hidden]
    t.update_model()
    torch.cuda.synchronize()
    recs = [int(b.bufs.record[0]) for b in opt.arena.buckets]
    print(step, "loss %.4f" % t.current_loss(), "gnorm", gn, "hid", hn, "w nan", bool(torch.isnan(opt.arena.weights).any()),
          "recs", recs[:3])
