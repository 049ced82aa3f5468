"""Static instruction mix of kernels in a hipcc -S assembly file.
usage: python tools/isa_mix.py file.s substring [substring ...]"""
import collections
import sys

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for line in s.split("\n"):
        if line.startswith("_Z") and line.split(":")[0].find(pat) >= 0 and ": ;" in line:
            name = line.split(":")[0]
            i = s.index(name + ": ;")
            j = s.index(".Lfunc_end", i)
            ops = collections.Counter()
            for ln in s[i:j].split("\n"):
                t = ln.strip().split()
                if t and not t[0].startswith((".", ";", "_")) and not t[0].endswith(":"):
                    ops[t[0]] += 1
            tot = sum(ops.values())
            valu = sum(v for k, v in ops.items() if k.startswith("v_"))
            pk = sum(v for k, v in ops.items() if k.startswith("v_pk_"))
            print(f"{name[:70]} total {tot} valu {valu} packed {pk} "
                  f"ds {sum(v for k, v in ops.items() if k.startswith('ds_'))}")
            for k, v in ops.most_common(18):
                print(f"   {k:28s} {v}")
