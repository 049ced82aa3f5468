"""U-Net (configs[4]) inference forms on the device, channels_last fp32, 256 chunks:
the eval model, its BatchNorm-folded copy (neural.fold_batchnorm) and that copy with every
conv + ReLU pair through torch.miopen_convolution_relu (bias + ReLU applied in the
convolution call). Prints ms per forward and the max |mask difference| to the eval model."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "real-time-audio-visual-zooming_amd")]
import torch
import torch.nn as nn
from avz import neural as N


class ConvReLU(nn.Module):
    def __init__(self, conv):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        c = self.conv
        return torch.miopen_convolution_relu(x, c.weight, c.bias, c.stride, c.padding,
                                             c.dilation, c.groups)


def fuse_relu(model):
    for seq in model.modules():
        if isinstance(seq, nn.Sequential):
            for i in range(len(seq) - 2):
                if (isinstance(seq[i], nn.Conv2d) and isinstance(seq[i + 1], nn.Identity)
                        and isinstance(seq[i + 2], nn.ReLU)):
                    seq[i] = ConvReLU(seq[i])
                    seq[i + 2] = nn.Identity()
    return model


dev = torch.device("cuda:0")
torch.manual_seed(0)
model = N.FreqPreservingUNet().eval().to(dev).to(memory_format=torch.channels_last)
x = torch.randn(256, 2, 513, 64, device=dev).contiguous(memory_format=torch.channels_last)


def t(fn, n=5):
    fn(); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3


with torch.no_grad():
    ref = model(x)
    print("eval model          %.1f ms / 256 chunks" % t(lambda: model(x)), flush=True)
    folded = N.fold_batchnorm(model)
    print("BN folded           %.1f ms, max diff %.2e" % (t(lambda: folded(x)), (folded(x) - ref).abs().max().item()), flush=True)
    fused = fuse_relu(N.fold_batchnorm(model))
    print("BN folded + convrelu %.1f ms, max diff %.2e" % (t(lambda: fused(x)), (fused(x) - ref).abs().max().item()), flush=True)
