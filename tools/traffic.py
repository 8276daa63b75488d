"""HBM traffic per launch of the stream kernel from the PMC passes written by
tools/profile.sh, corrected with the calibration passes of
tools/micro/fetch_calib (a kernel streaming a known byte count with the same
16-byte-per-lane pattern).  Writes profiles/traffic_latest.json (read by
bench.py as roofline.traffic).

    python tools/traffic.py PROFILE_DIR [OUT_JSON]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402

CALIB_BYTES = 512 << 20   # tools/micro/fetch_calib.hip


def main():
    d = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "traffic_latest.json")
    res = summarise(d)
    # the headline's stream kernel: the in-kernel QN variant (its last
    # template argument true) when the run launched it, else the first one
    fbs = [k for k in res if k.startswith("fbs_kernel")]
    kern = next((k for k in fbs if k.replace(" ", "").endswith(",true>")), fbs[0])
    fetch_kib = res[kern]["FETCH_SIZE"]
    write_kib = res[kern]["WRITE_SIZE"]
    cal_r = res["stream_read"]["FETCH_SIZE"] * 1024.0
    cal_w = res["stream_write"]["WRITE_SIZE"] * 1024.0
    fr, fw = CALIB_BYTES / cal_r, CALIB_BYTES / cal_w
    rec = {
        "kernel": kern,
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "calibration": {
            "kernel": "tools/micro/fetch_calib.hip: 512 MiB streamed with 16-byte-per-lane loads / stores",
            "known_bytes": CALIB_BYTES,
            "fetch_size_bytes": cal_r,
            "write_size_bytes": cal_w,
            "read_factor": fr,
            "write_factor": fw,
        },
        "hbm_bytes_per_launch": fetch_kib * 1024.0 * fr + write_kib * 1024.0 * fw,
        "source": os.path.abspath(d),
    }
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
