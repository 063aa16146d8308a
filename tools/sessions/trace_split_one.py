import os, sys, zlib
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
os.environ["ZCRC_SPLIT_TRACE"] = "1"
import torch, inflate_streams as S, zipsfs_amd as z
for kind in ("text", "spectrum"):
    data = S.PAYLOADS[kind](1 << 20, 77)
    comp = S.deflate(data, 6)
    src = torch.frombuffer(bytearray(comp), dtype=torch.uint8).to("cuda:0")
    dst = torch.empty(len(data), dtype=torch.uint8, device="cuda:0")
    ol, st = z.inflate_device(src, dst)
    torch.cuda.synchronize()
    print(kind, int(st.item()), int(ol.item()), bytes(dst.cpu().numpy()) == data, flush=True)
