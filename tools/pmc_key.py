"""PMC entry keys of profiles/pmc_traffic.json: a bench config plus every layout option that
differs from its default, e.g. "zipf", "zipf@ia8,oa8", "zipf@oa1", "4k@os4352".

bench.py looks its roofline.traffic / valu entry up by this key (so a layout never borrows the
default layout's counters), and tools/gpu_traffic.sh / gpu_valu.sh / gpu_stall.sh accept keys as
config tokens and run bench.py with the matching arguments:

  python tools/pmc_key.py args zipf@ia8,oa8   ->  --config zipf --in-align 8 --out-align 8
  python tools/pmc_key.py base zipf@ia8,oa8   ->  zipf
  python tools/pmc_key.py file zipf@ia8,oa8   ->  zipf_ia8_oa8   (a file-name-safe form)"""
import sys

# short name -> (bench.py option, default)
OPTS = {"ia": ("--in-align", 64), "oa": ("--out-align", 128), "seg": ("--seg-blocks", 128),
        "is": ("--in-stride", 0), "os": ("--out-stride", 0), "ps": ("--plain-stride", 0)}
ZIPF_ONLY = ("ia", "oa", "seg")


def key(config, **vals):
    """vals: short name -> value (bench.py's parsed options)"""
    parts = []
    for short, (_, default) in OPTS.items():
        if short in ZIPF_ONLY and not config.startswith("zipf"):
            continue
        v = vals.get(short, default)
        if v != default:
            parts.append(f"{short}{v}")
    return config + ("@" + ",".join(parts) if parts else "")


def key_from_args(args):
    return key(args.config, ia=args.in_align, oa=args.out_align, seg=args.seg_blocks, **{
        "is": args.in_stride, "os": args.out_stride, "ps": args.plain_stride})


def parse(k):
    config, _, rest = k.partition("@")
    vals = {}
    for p in filter(None, rest.split(",")):
        short = next(s for s in sorted(OPTS, key=len, reverse=True) if p.startswith(s))
        vals[short] = int(p[len(short):])
    return config, vals


def bench_args(k):
    config, vals = parse(k)
    out = ["--config", config]
    for short, v in vals.items():
        out += [OPTS[short][0], str(v)]
    return out


def file_safe(k):
    return k.replace("@", "_").replace(",", "_")


if __name__ == "__main__":
    what, k = sys.argv[1], sys.argv[2]
    if what == "args":
        print(" ".join(bench_args(k)))
    elif what == "base":
        print(parse(k)[0])
    else:
        print(file_safe(k))
