"""Print the kernel timeline of one graph-replay step from a rocprofv3
kernel trace (csv): python tools/prof_step.py gpurun_out/prof_kt/kt_kernel_trace.csv [k]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts with its batch load (pool_copy_k) when the bench loads in-graph,
# else with its ego-net build
# (the largest pool copy: the fine-tune bench also copies its targets in one)
copies = [(i, int(r["Grid_Size_X"])) for i, r in enumerate(rows) if "pool_copy_k" in r["Kernel_Name"]]
gmax = max((gsz for _, gsz in copies), default=0)
starts = [i for i, gsz in copies if gsz == gmax]
if len(starts) < 3:
    starts = [i for i, r in enumerate(rows) if "egonet_" in r["Kernel_Name"] and ("count_k" in r["Kernel_Name"] or "onepass_k" in r["Kernel_Name"])]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
i0, i1 = starts[k], starts[k + 1]
t0 = int(rows[i0]["Start_Timestamp"])
last = 0
for r in rows[i0:i1]:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].replace("void ", "").replace("scgib::", "")
    if "at::" in name:  # a torch kernel: its functor says which op it is
        name = name.split("(")[0][:150]
    else:
        name = name.split("(")[0].split("<")[0][:48]
    print(f"{s/1000:8.2f} {e/1000:8.2f} {(e-s)/1000:7.2f} gap{(s-last)/1000:7.2f} "
          f"q{r['Queue_Id']} {name} g{r['Grid_Size_X']}")
    last = max(last, e)
print("span", (int(rows[i1]["Start_Timestamp"]) - t0) / 1000)
