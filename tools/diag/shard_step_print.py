import json, sys
for line in open(sys.argv[1]):
    if line[:2] in ("1 ", "2 ", "4 ", "8 "):
        N, js = line.split(" ", 1); d = json.loads(js)
        print(N, round(d["max_wall_ms_pipelined"], 2), [round(r["wall_ms_pipelined"], 2) for r in d["ranks"]], [r["tie_rows"] for r in d["ranks"]])
