import sys, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from iclr_17_compression_amd import kernels, synth
from iclr_17_compression_amd.model import ImageCompressor
N, B, H, W = 192, 1, 64, 64
dev = 'cuda'
net = ImageCompressor(out_channel_N=N)
net.load_state_dict({k: torch.from_numpy(v) for k, v in synth.trained_like_state_dict(N, 1).items()})
net = net.to(dev).eval()
s2 = torch.from_numpy(synth.normal_like(21, (B, N, H // 4, W // 4), 0.6))
F = torch.nn.functional
sd = net.state_dict()
with torch.no_grad():
    ref = F.conv_transpose2d(s2, sd["Decoder.deconv3.weight"].cpu(), sd["Decoder.deconv3.bias"].cpu(), stride=4, padding=4, output_padding=3)
    d3 = net.Decoder.packed()[2]
    hs = kernels.split_planes(s2.permute(0, 2, 3, 1).contiguous().to(dev))
    _, r1, _ = kernels.deconv3_x6(hs, d3, net.Decoder.deconv3.bias, want_recon=True)
    _, r2, _ = kernels.deconv3_x6(hs, d3, net.Decoder.deconv3.bias, want_recon=True, w_split=net.Decoder.packed_deconv3_x6())
    torch.cuda.synchronize()
    r1, r2 = r1.cpu(), r2.cpu()
    for name, r in (("skip", r1), ("pre", r2)):
        e = (r - ref).abs()
        print(name, "max err", e.max().item())
        for co in range(3):
            row = []
            for ry in range(4):
                row.append(" ".join(f"{e[0, co, ry::4, rx::4].max().item():.1e}" for rx in range(4)))
            print("  co", co, " | ".join(row))
