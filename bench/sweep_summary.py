import json, sys
for r in json.load(open(sys.argv[1])):
    print(r["shape"], {k.replace("_tflops_median","").replace("kgs_",""):v for k,v in r.items() if k.endswith("median")}, set(r["rel_err_vs_hipblaslt"].values()))
