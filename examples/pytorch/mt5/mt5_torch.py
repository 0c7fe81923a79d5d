"""The same mT5 training in eager PyTorch, the reference's baseline
(examples/python/pytorch/mt5/mt5_torch.py; synthetic data, random weights)."""
import os
import sys
import time

import torch
from mt5_ff import mt5_config, synthetic_data
from transformers import MT5ForConditionalGeneration


def main():
    quick = "FF_EXAMPLE_SAMPLES" in os.environ
    device = "cuda" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(42)
    model = MT5ForConditionalGeneration(mt5_config(quick)).to(device)
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 1024))
    seq = 16 if quick else 48
    bs = int(sys.argv[sys.argv.index("-b") + 1]) if "-b" in sys.argv else 8
    ids, mask, y_ids, labels = (torch.as_tensor(a) for a in synthetic_data(n, seq, seq, model.config.vocab_size))
    opt = torch.optim.SGD(model.parameters(), lr=0.01)
    t0 = time.time()
    steps = n // bs
    for i in range(steps):
        sl = slice(i * bs, (i + 1) * bs)
        out = model(input_ids=ids[sl].to(device), attention_mask=mask[sl].to(device),
                    decoder_input_ids=y_ids[sl].to(device), labels=labels[sl].long().to(device), use_cache=False)
        opt.zero_grad()
        out.loss.backward()
        opt.step()
        if i % 10 == 0:
            print(f"step {i}: loss {out.loss.item():.4f}")
    el = time.time() - t0
    print("ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" % (el, steps * bs / el))


if __name__ == "__main__":
    main()
