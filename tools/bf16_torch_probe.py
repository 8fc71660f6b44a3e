"""torch's own hipBLASLt: bf16 x bf16 GEMMs (bf16 or fp32 out) and the fp32 -> bf16 cast they need, on the
PDVC step's dominant shapes (MI355X)."""
import torch

def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps

for (M, N, K, tb) in [(245760, 512, 512, True), (245760, 512, 512, False), (53248, 5748, 512, True),
                      (53248, 2048, 1536, True)]:
    a = torch.randn(M, K, device='cuda')
    w = torch.randn((N, K) if tb else (K, N), device='cuda')
    B = w.t() if tb else w
    ab, Bb = a.bfloat16(), B.bfloat16()
    fl = 2 * M * N * K
    ms32 = t(lambda: torch.mm(a, B))
    mscast = t(lambda: a.to(torch.bfloat16))
    ms16 = t(lambda: torch.mm(ab, Bb))
    try:
        ms16f = t(lambda: torch.mm(ab, Bb, out_dtype=torch.float32))
    except Exception as e:
        ms16f = float('nan'); print(e)
    print(f"{M}x{N}x{K} tb={tb}: fp32 {fl/ms32/1e9:.0f} TF/s ({ms32:.3f} ms); cast A {mscast:.3f} ms; "
          f"bf16->bf16 {fl/ms16/1e9:.0f} TF/s ({ms16:.3f} ms); bf16->fp32 {fl/ms16f/1e9:.0f} TF/s ({ms16f:.3f} ms)",
          flush=True)
wg = torch.randn(245760, 512, device='cuda'); xg = torch.randn(245760, 512, device='cuda')
wgb, xgb = wg.bfloat16(), xg.bfloat16()
fl = 2 * 512 * 512 * 245760
print(f"wgrad 512x512x245760: fp32 {fl/t(lambda: wg.t() @ xg)/1e9:.0f} TF/s; bf16->fp32 "
      f"{fl/t(lambda: torch.mm(wgb.t(), xgb, out_dtype=torch.float32))/1e9:.0f} TF/s")
