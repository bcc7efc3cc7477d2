"""Extract the reference's own sample data into tests/golden/reference/ (run
here, where /root/reference exists; the outputs are committed data):

* the JSON bodies of the /api/v1/export responses and the /api/v1/import
  request in simulator/docs/api-samples/v1/{export,import}.md;
* the web UI's object templates web/components/lib/templates/*.yaml, as JSON.

Only data is written (documents and object templates), never source."""
import json
import os
import re
import sys

import yaml

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "reference")


def bodies(md_path):
    text = open(md_path).read()
    out = []
    for block in re.findall(r"```\n(.*?)```", text, re.S):
        i = block.find("\n{")
        if i >= 0:
            out.append(json.loads(block[i + 1:].strip()))
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    docs = os.path.join(REF, "simulator/docs/api-samples/v1")
    for k, doc in enumerate(bodies(os.path.join(docs, "export.md"))):
        json.dump(doc, open(os.path.join(OUT, f"export_case{k + 1}.json"), "w"), indent=1, sort_keys=True)
    for k, doc in enumerate(bodies(os.path.join(docs, "import.md"))):
        json.dump(doc, open(os.path.join(OUT, f"import_case{k + 1}.json"), "w"), indent=1, sort_keys=True)
    tdir = os.path.join(REF, "web/components/lib/templates")
    for f in sorted(os.listdir(tdir)):
        if f.endswith(".yaml"):
            obj = yaml.safe_load(open(os.path.join(tdir, f)))
            json.dump(obj, open(os.path.join(OUT, "template_" + f[:-5] + ".json"), "w"), indent=1, sort_keys=True)
    print("\n".join(sorted(os.listdir(OUT))))


if __name__ == "__main__":
    sys.exit(main())
