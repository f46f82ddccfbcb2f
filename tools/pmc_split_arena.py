import csv, json, sys, collections
for i in (1, 2, 3, 4):
    d = f"gpurun_out/r06o/pmc{i}"
    seq = json.loads(open(f"gpurun_out/r06o/pmc{i}.json").read())["seq"]
    rows = list(csv.DictReader(open(f"{d}/pmc_counter_collection.csv")))
    by = collections.defaultdict(dict)
    for r in rows:
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        by[int(r["Dispatch_Id"])]["_t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ids = sorted(by)[-24:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (a, ms), di in zip(seq, ids):
        for k, v in by[di].items():
            agg[a][k].append(v)
    print("pass", i)
    for a in "AB":
        print(" ", a, {k: round(sum(v) / len(v), 4 if k == "_t" else 0) for k, v in sorted(agg[a].items())})
