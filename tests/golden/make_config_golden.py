"""Regenerates config_cases.json from the REAL reference NetworkConfig.

Runs oracle/_ref/ref_config_driver (the reference's own config.cpp compiled
where it lies under /root/reference by `make -C oracle ref`) on every case
below and stores input text + output.  Only run in the build container;
the committed JSON is what tests read (the GPU box has no /root/reference).
"""
import json
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
DRIVER = REPO / "oracle" / "_ref" / "ref_config_driver"

NETWORK_TXT = "".join(f"192.168.1.{100 + i}:{8000 + i}\n" for i in range(20))

CASES = {
    "network_txt": NETWORK_TXT,
    "one_seed": "127.0.0.1:6000\n",
    "three_seeds_params": "# seeds\n127.0.0.1:6000\n 127.0.0.1:6001 \n\n127.0.0.1:6002\nping_interval=7\nmessage_interval = 2\nmax_messages=4\nmax_missed_pings=5\n",
    "unknown_key_ignored": "10.0.0.1:1\nfoo=bar\n",
    "crlf_lines": "10.0.0.1:7000\r\n10.0.0.2:7001\r\n",
    "lenient_stoi_port": "10.0.0.1:8000abc\n",
    "bad_ip": "300.1.1.1:8000\n",
    "bad_port_range": "10.0.0.1:70000\n",
    "bad_port_zero": "10.0.0.1:0\n",
    "bad_port_text": "10.0.0.1:abc\n",
    "missing_port": "10.0.0.1:\n",
    "no_separator": "justtext\n",
    "empty_key": "=5\n10.0.0.1:1\n",
    "empty_value": "ping_interval=\n10.0.0.1:1\n",
    "non_numeric_value": "10.0.0.1:1\nping_interval=abc\n",
    "no_seeds": "# nothing\nping_interval=3\n",
    "duplicate_seeds": "10.0.0.1:1\n10.0.0.1:1\n",
    "negative_interval": "10.0.0.1:1\nping_interval=-1\n",
    "zero_max_messages": "10.0.0.1:1\nmax_messages=0\n",
    "comment_and_blank_only_then_seed": "\n\n# c\n   \n10.0.0.9:9\n",
    "line_number_in_error": "10.0.0.1:1\n10.0.0.2:2\nbogus\n",
}


def main():
    if not DRIVER.exists():
        sys.exit(f"{DRIVER} missing: run `make -C oracle ref` (needs /root/reference)")
    out = {"source": "reference config.cpp via oracle/_ref/ref_config_driver (NetworkConfig::NetworkConfig)",
           "cases": []}
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for name, text in CASES.items():
            p = Path(td) / f"{name}.txt"
            p.write_bytes(text.encode())
            paths.append(p)
        missing = str(Path(td) / "does_not_exist.txt")
        res = subprocess.run([str(DRIVER)] + [str(p) for p in paths] + [missing], capture_output=True, text=True,
                             check=True)
        lines = res.stdout.strip().split("\n")
        names = list(CASES) + ["missing_file"]
        texts = list(CASES.values()) + [None]
        for name, text, line in zip(names, texts, lines):
            rec = json.loads(line)
            if name == "missing_file":
                rec["what"] = rec["what"].replace(missing, "<PATH>")
            out["cases"].append({"name": name, "text": text, "result": rec})
    (HERE / "config_cases.json").write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
