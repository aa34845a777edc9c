"""Compare two bench.py --rows-out files (steps x global batch x 14): equal bit for bit?"""
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
print(f"{sys.argv[1]}: world {a['world']}, global batch {a['global_batch']}, steps {a['steps']}")
print(f"{sys.argv[2]}: world {b['world']}, global batch {b['global_batch']}, steps {b['steps']}")
ra, rb = a["rows"], b["rows"]
assert ra.shape == rb.shape, (ra.shape, rb.shape)
eq = torch.equal(ra, rb)
print("rows bit-identical:", eq, "" if eq else f"max |diff| {float((ra - rb).abs().max()):.3e}")
sys.exit(0 if eq else 1)
