import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
acc = [r for r in rows if "k_accumulate" in r["Kernel_Name"]]
t0 = int(acc[8]["Start_Timestamp"]) - 500000  # second batch
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0: continue
    n = r["Kernel_Name"].split("(")[0].replace("void ","").replace("mbls::","")[:34]
    if any(k in n for k in ("k_accumulate", "k_bucket_small", "k_reduce_scaled", "k_final", "k_digits_part", "k_part_sort", "k_jac")):
        print(f"{(s-t0)/1e3:9.1f} {(e-s)/1e3:8.1f} q{r.get('Queue_Id','?'):>3} {n}")
