"""RssAnon (MiB) after each step of tests/test_gpu_parity.py
test_config_c2_c3_full_size, to find the step that keeps ~10 GiB of anonymous
host memory resident (profiles/r05/r05_rss_probe.txt)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "isa-l_amd"))

import ecutil  # noqa: E402
import isal_amd as engine  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def anon(tag):
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("RssAnon"):
                print(tag, int(line.split()[1]) // 1024, flush=True)


def main():
    gpu = torch.device("cuda:0")
    oracle = ecutil.oracle()
    anon("start")
    k, p, n, ns = 10, 4, 1 << 20, 1024
    a = engine.gf_gen_rs_matrix(k + p, k)
    data, coding, dptr, cptr = T._stripes(torch, gpu, ns, k, p, n, 2024)
    torch.cuda.synchronize()
    anon("stripes")
    enc = engine.Batch(n, k, p, engine.ec_init_tables(k, p, a[k * k:]), ns, dptr, cptr)
    anon("batch")
    enc.encode(0)
    torch.cuda.synchronize()
    anon("encode")
    T._check_stripes_vs_oracle(oracle, a[k * k:], k, p, lambda s: [data[s, j] for j in range(k)], coding, 64)
    anon("check 64 stripes")
    errs = [4, 6, 7]
    ret, c, surv = ecutil.decode_matrix(a, k, errs)
    anon("decode matrix")
    frag = lambda s, i: data[s, i] if i < k else coding[s, i - k]  # noqa: E731
    rec = torch.zeros((ns, len(errs), n), dtype=torch.uint8, device=gpu)
    sptr = [int(frag(s, i).data_ptr()) for s in range(ns) for i in surv]
    rptr = [int(rec[s, i].data_ptr()) for s in range(ns) for i in range(len(errs))]
    anon("decode pointers")
    dec = engine.Batch(n, k, len(errs), engine.ec_init_tables(k, len(errs), c), ns, sptr, rptr)
    dec.encode(0)
    torch.cuda.synchronize()
    anon("decode")
    T._check_stripes_vs_oracle(oracle, c, k, len(errs), lambda s: [frag(s, i) for i in surv], rec, 64)
    anon("check decode 64 stripes")
    sel = data[:, errs]
    anon("data[:, errs]")
    eq = bool(torch.equal(rec, sel))
    anon(f"torch.equal {eq}")
    dec.close()
    enc.close()
    del data, coding
    anon("freed")


if __name__ == "__main__":
    main()
