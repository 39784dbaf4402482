import math, torch, sys
sys.path.insert(0, '.')
from tests.test_decode_gpu import _setup_cache, _bf
from kgs.ops.decode import PagedKVCache, paged_decode_attention, ref_cache_write, ref_paged_decode
torch.manual_seed(0)
heads, hkv = 32, 8
for ctxs in ([1, 31, 32, 77, 300], [300], [64], [33]):
    b = len(ctxs)
    cache = PagedKVCache(1, 64, hkv, 'cuda')
    bt = _setup_cache(b, ctxs, hkv, 64).to('cuda')
    for i, c in enumerate(ctxs):
        pos = torch.arange(c, device='cuda')
        slots = (bt[i, pos // 32].long() * 32 + pos % 32).int()
        ref_cache_write(cache.layer(0), _bf(c, hkv, 128), _bf(c, hkv, 128), slots)
    q = _bf(b, heads * 128)
    ctx_t = torch.tensor(ctxs, dtype=torch.int32, device='cuda')
    ref = ref_paged_decode(q, cache.layer(0), bt, ctx_t, heads, hkv)
    for pps in (100, 1, 2, 3, None):
        o = paged_decode_attention(q, cache.layer(0), bt, ctx_t, heads, hkv, pages_per_split=pps)
        torch.cuda.synchronize()
        err = (o.float() - ref).abs().amax(-1)
        print(ctxs, pps, [round(e, 3) for e in err.tolist()], flush=True)
