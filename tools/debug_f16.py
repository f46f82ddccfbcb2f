"""Print the elements where the HIP engine and the C oracle disagree for one fp16 case."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import orc
from fedml_amd.engine import get_engine
eng = get_engine(0)
for (K, P, mode) in [(3, 1023, 0), (5, 4096 * 8 + 3, 0), (3, 1023, 2), (3, 1023, 1)]:
    g = torch.Generator().manual_seed(K * 1000 + P)
    xs = [torch.randn((P,), generator=g, dtype=torch.float64).to(torch.float16) for _ in range(K)]
    counts = [int(v) for v in torch.randint(50, 601, (K,), generator=g)]
    N = sum(counts)
    coef = [c / N for c in counts] if mode == 0 else counts
    exp = orc.weighted_sum(xs, mode, coef, float(N))
    got = eng.weighted_sum([x.cuda() for x in xs], mode, coef, float(N)).cpu()
    gb, eb = got.view(torch.int16), exp.view(torch.int16)
    bad = torch.nonzero(gb != eb).reshape(-1)
    print(f"K={K} P={P} mode={mode}: {bad.numel()} mismatches")
    for i in bad[:8].tolist():
        print("  e", i, "x", [hex(x[i].view(torch.int16).item() & 0xffff) for x in xs], [float(x[i]) for x in xs],
              "got", hex(gb[i].item() & 0xffff), float(got[i]), "exp", hex(eb[i].item() & 0xffff), float(exp[i]),
              "coef", coef)
