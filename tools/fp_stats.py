import csv, glob
f = glob.glob("/tmp/fp/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(float(r["MinNs"]) / 1e3, 1))
f = glob.glob("/tmp/fp/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f))]
chain = rows[-5:]
print([(r["Kernel_Name"][:30], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) // 1000) for r in chain])
print("chain span us", (int(chain[-1]["End_Timestamp"]) - int(chain[0]["Start_Timestamp"])) / 1000)
