"""Which dtype does nn.LSTM compute in under bf16 autocast on ROCm (MIOpen)?"""
import torch

from gaussiank_sgd_amd.models.lstm_ptb import PTBLSTM

m = PTBLSTM(batch_size=4).cuda()
x = torch.randint(0, 10000, (35, 4), device="cuda")
with torch.autocast("cuda", dtype=torch.bfloat16):
    e = m.word_embeddings(x)
    o, h = m.lstm(e, m.init_hidden(4))
print("embedding", e.dtype, "lstm out", o.dtype, "h", h[0].dtype, "cudnn", torch.backends.cudnn.enabled)
