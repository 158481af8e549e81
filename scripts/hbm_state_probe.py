"""The box's HBM "state" over time (r06: one box measured the encode's byte mix at 3.37 ms early in a
call and 3.75 ms minutes later -- the "fast / slow box types" of r03-r05).  Alternates: the
box-ceiling probe (libtecprobe, min of 3) with the hwmon sensors of the GPU's PCI function (edge /
junction / memory temperature, power), then `--load-s` seconds of encode load, then an idle gap;
prints one JSON line per sample.  Measurement only.
    python scripts/hbm_state_probe.py --samples 12 --load-s 8 --idle-s 0
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sensors(torch, dev):
    out = {}
    try:
        p = torch.cuda.get_device_properties(dev)
        base = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        for h in glob.glob(os.path.join(base, "hwmon", "hwmon*")):
            for f in glob.glob(os.path.join(h, "temp*_input")):
                lab = f.replace("_input", "_label")
                name = open(lab).read().strip() if os.path.exists(lab) else os.path.basename(f)
                out["temp_" + name] = int(open(f).read()) / 1000.0
            for f in glob.glob(os.path.join(h, "power*_average")) + glob.glob(os.path.join(h, "power*_input")):
                out[os.path.basename(f)] = int(open(f).read()) / 1e6
        for key, fn in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk")):
            try:
                cur = [l for l in open(os.path.join(base, fn)).read().split("\n") if l.strip().endswith("*")]
                out[key] = cur[0].strip() if cur else None
            except OSError:
                pass
    except Exception as e:
        out["error"] = str(e)[:80]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=12)
    ap.add_argument("--load-s", type=float, default=8.0)
    ap.add_argument("--idle-s", type=float, default=0.0)
    args = ap.parse_args()
    import torch
    import bench
    import tape_amd as T
    from tape_amd import batch
    dev = torch.device("cuda", 0)
    L, nobj = 4 << 20, 1024
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = 20 * g.slice_len
    d_in = torch.empty(nobj * L, dtype=torch.uint8, device=dev)
    bench.splitmix_fill(torch, d_in, 0, nobj, L)
    d_out = torch.empty(nobj * per, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(nobj)])
    alg = bench.ALG_BYTES["encode"] * nobj
    t0 = time.time()
    for k in range(args.samples):
        c = bench.box_ceiling(torch, d_in, nobj * L, d_out, nobj * per, stream, alg)
        # the encode kernel's own time right after the probe
        batch.kernel_time_ms()
        batch.kernel_timing(True)
        for _ in range(5):
            batch.encode_batch(s, d_in, objs, d_out, stream)
        torch.cuda.synchronize()
        batch.kernel_timing(False)
        kms, _ = batch.kernel_time_ms()
        print(json.dumps({"t_s": round(time.time() - t0, 1), "blocks_ms": c.get("blocks_ms"), "rows_ms": c.get("rows_ms"),
                          "encode_ms": round(kms / 5, 4), **sensors(torch, dev)}), flush=True)
        t = time.time()
        while time.time() - t < args.load_s:
            batch.encode_batch(s, d_in, objs, d_out, stream)
            torch.cuda.synchronize()
        if args.idle_s:
            time.sleep(args.idle_s)


if __name__ == "__main__":
    main()
