"""Regenerate tests/golden/nba.json — the NBA dataset of the reference GoTest suite.

Reads the data literals of src/graph/test/TraverseTestBase.h (players_ :314-380, teams_
:382-416, the serve/like/teammate chains of initData() :500-806) as TEXT and writes them as JSON.
Vertex ids are std::hash<std::string>(name) (TraverseTestBase.h:122-126), computed by the test
side. Run here only (the reference is not present on the GPU box):

    python tests/golden/make_nba.py /root/reference
"""
import json
import os
import re
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = open(os.path.join(ref, "src/graph/test/TraverseTestBase.h")).read()

players, seen = [], set()
for name, age in re.findall(r'Player\{"([^"]+)",\s*(\d+)', src):
    if name not in seen:                      # VertexHolder::emplace keeps the first
        seen.add(name)
        players.append([name, int(age)])
teams, tseen = [], set()
for name in re.findall(r'Team\{"([^"]+)"\}', src):
    if name not in tseen:
        tseen.add(name)
        teams.append(name)

serve, like, teammate = [], [], []
init = src[src.index("AssertionResult TraverseTestBase::initData()"):src.index("AssertionResult TraverseTestBase::prepareData()")]
for block in re.findall(r'players_\["([^"]+)"\]((?:\s*\.\w+\([^)]*\))+)\s*;', init):
    who, chain = block
    for meth, args in re.findall(r'\.(\w+)\(([^)]*)\)', chain):
        a = [x.strip() for x in args.split(",")]
        if meth == "serve":
            serve.append([who, a[0].strip('"'), int(a[1]), int(a[2]), int(a[3])])
        elif meth == "like":
            like.append([who, a[0].strip('"'), int(a[1])])
        elif meth == "teammate":
            teammate.append([who, a[0].strip('"'), int(a[1]), int(a[2])])
        else:
            raise SystemExit(f"unknown method {meth}")

out = {"source": "src/graph/test/TraverseTestBase.h", "space_parts": 1,
       "tag_ids": {"player": 2, "team": 3, "bachelor": 7},
       "edge_types": {"serve": 4, "like": 5, "teammate": 6},
       "players": players, "teams": teams, "serve": serve, "like": like, "teammate": teammate}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nba.json")
with open(path, "w") as f:
    json.dump(out, f, indent=0)
print(f"wrote {path}: {len(players)} players, {len(teams)} teams, {len(serve)} serve, "
      f"{len(like)} like, {len(teammate)} teammate")
