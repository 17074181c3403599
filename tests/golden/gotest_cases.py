"""Known answers transcribed from the reference GoTest suite (src/graph/test/GoTest.cpp) on the
NBA fixture (tests/golden/nba.json). Data only: queries and expected rows.

Placeholders: {P:<name>} / {T:<name>} in a query are replaced by the player / team vid
(std::hash<std::string>(name), TraverseTestBase.h:122-126); "P:<name>" / "T:<name>" in an
expected row stand for that vid. Rows are compared sorted, as verifyResult does
(src/graph/test/TestBase.h:188-233). "empty": the response had no rows. "ok_only": the reference only
asserts that the query succeeds (its rows are then compared with the oracle's).
"""

RK = ("T:Mavericks",), ("T:Kings",), ("T:Bulls",)
MTON_PROPS = [("P:Manu Ginobili", 95, "Manu Ginobili"), ("P:LaMarcus Aldridge", 90, "LaMarcus Aldridge"),
              ("P:Tim Duncan", 95, "Tim Duncan"), ("P:Tony Parker", 95, "Tony Parker"),
              ("P:Tony Parker", 75, "Tony Parker"), ("P:Tim Duncan", 75, "Tim Duncan"),
              ("P:Tim Duncan", 90, "Tim Duncan")]
MTON_REV = [("P:Tim Duncan",), ("P:LaMarcus Aldridge",), ("P:Marco Belinelli",), ("P:Boris Diaw",),
            ("P:Dejounte Murray",), ("P:Tony Parker",), ("P:Manu Ginobili",), ("P:Danny Green",),
            ("P:Aron Baynes",), ("P:Tiago Splitter",), ("P:Shaquile O'Neal",), ("P:Rudy Gay",),
            ("P:Damian Lillard",)]
MTON_SPURS = [("P:" + n,) for n in (
    "Tim Duncan", "Tony Parker", "Manu Ginobili", "LaMarcus Aldridge", "Rudy Gay", "Marco Belinelli",
    "Danny Green", "Kyle Anderson", "Aron Baynes", "Boris Diaw", "Tiago Splitter", "Cory Joseph", "David West",
    "Jonathon Simmons", "Dejounte Murray", "Tracy McGrady", "Paul Gasol", "Marco Belinelli")]
MTON_BI = MTON_REV + [("P:" + n,) for n in (
    "LeBron James", "Russell Westbrook", "Chris Paul", "Kyle Anderson", "Kevin Durant", "James Harden")]
MTON_STAR = [("T:Thunders", 0), (0, "P:Paul George"), (0, "P:James Harden"), ("T:Pacers", 0), ("T:Thunders", 0),
             (0, "P:Russell Westbrook"), ("T:Thunders", 0), ("T:Rockets", 0), (0, "P:Russell Westbrook")]
MTON_STAR_PROPS = [("T:Thunders", 0, 2008, 0, ""), (0, "P:Paul George", 0, 90, "Paul George"),
                   (0, "P:James Harden", 0, 90, "James Harden"), ("T:Pacers", 0, 2010, 0, ""),
                   ("T:Thunders", 0, 2017, 0, ""), (0, "P:Russell Westbrook", 0, 95, "Russell Westbrook"),
                   ("T:Thunders", 0, 2009, 0, ""), ("T:Rockets", 0, 2012, 0, ""),
                   (0, "P:Russell Westbrook", 0, 80, "Russell Westbrook")]

# NStepQueryHangAndOOM (GoTest.cpp:3069-3107): GO 1 TO 3 STEPS FROM Tim Duncan OVER like, 11 rows
NSTEP_HANG = [("P:" + n,) for n in (
    "Tony Parker", "Manu Ginobili", "Tim Duncan", "Tim Duncan", "LaMarcus Aldridge", "Manu Ginobili",
    "Tony Parker", "Manu Ginobili", "Tim Duncan", "Tim Duncan", "Tony Parker")]

CASES = [
    # OneStepOutBound (GoTest.cpp:35-168)
    dict(line=37, query="GO FROM {P:Tim Duncan} OVER serve", rows=[("T:Spurs",)]),
    dict(line=63, query="GO FROM {P:Boris Diaw} OVER serve YIELD $^.player.name, serve.start_year, "
                        "serve.end_year, $$.team.name",
         rows=[("Boris Diaw", 2003, 2005, "Hawks"), ("Boris Diaw", 2005, 2008, "Suns"),
               ("Boris Diaw", 2008, 2012, "Hornets"), ("Boris Diaw", 2012, 2016, "Spurs"),
               ("Boris Diaw", 2016, 2017, "Jazz")]),
    dict(line=84, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year >= 2013 && "
                        "serve.end_year <= 2018 YIELD $^.player.name, serve.start_year, serve.end_year, "
                        "$$.team.name",
         rows=[("Rajon Rondo", 2014, 2015, "Mavericks"), ("Rajon Rondo", 2015, 2016, "Kings"),
               ("Rajon Rondo", 2016, 2017, "Bulls"), ("Rajon Rondo", 2017, 2018, "Pelicans")]),
    # OneStepInBound (:247-265)
    dict(line=249, query="GO FROM {T:Thunders} OVER serve REVERSELY",
         rows=[("P:Russell Westbrook",), ("P:Kevin Durant",), ("P:James Harden",), ("P:Carmelo Anthony",),
               ("P:Paul George",), ("P:Ray Allen",)]),
    # Distinct (:294-341)
    dict(line=297, query="GO FROM {P:Nobody} OVER serve YIELD DISTINCT $^.player.name as name, "
                         "$$.team.name as name", empty=True),
    dict(line=329, query="GO 2 STEPS FROM {P:Tony Parker} OVER like YIELD DISTINCT like._dst",
         rows=[(3394245602834314645,), (-7579316172763586624,), (5662213458193308137,)]),
    # MULTI_EDGES (:435-...)
    dict(line=439, query="GO FROM {P:Russell Westbrook} OVER serve, like",
         rows=[("T:Thunders", 0), (0, "P:Paul George"), (0, "P:James Harden")]),
    dict(line=452, query="GO FROM {P:Russell Westbrook} OVER serve, like REVERSELY "
                         "YIELD serve._dst, like._dst, serve._type, like._type",
         rows=[(0, "P:James Harden", 0, -5), (0, "P:Dejounte Murray", 0, -5), (0, "P:Paul George", 0, -5)]),
    # ReverselyOneStep (:1094-1170)
    dict(line=1097, query="GO FROM hash('Tim Duncan') OVER like REVERSELY YIELD like._dst",
         rows=[("P:Tony Parker",), ("P:Manu Ginobili",), ("P:LaMarcus Aldridge",), ("P:Marco Belinelli",),
               ("P:Danny Green",), ("P:Aron Baynes",), ("P:Boris Diaw",), ("P:Tiago Splitter",),
               ("P:Dejounte Murray",), ("P:Shaquile O'Neal",)]),
    dict(line=1117, query="GO FROM hash('Tim Duncan') OVER * REVERSELY YIELD like._dst",
         rows=[("P:Tony Parker",), ("P:Manu Ginobili",), ("P:LaMarcus Aldridge",), ("P:Marco Belinelli",),
               ("P:Danny Green",), ("P:Aron Baynes",), ("P:Boris Diaw",), ("P:Tiago Splitter",),
               ("P:Dejounte Murray",), ("P:Shaquile O'Neal",), (0,), (0,)]),
    dict(line=1139, query="GO FROM hash('Tim Duncan') OVER like REVERSELY YIELD $$.player.name",
         rows=[("Tony Parker",), ("Manu Ginobili",), ("LaMarcus Aldridge",), ("Marco Belinelli",),
               ("Danny Green",), ("Aron Baynes",), ("Boris Diaw",), ("Tiago Splitter",),
               ("Dejounte Murray",), ("Shaquile O'Neal",)]),
    dict(line=1157, query="GO FROM hash('Tim Duncan') OVER like REVERSELY WHERE $$.player.age < 35 "
                          "YIELD $$.player.name",
         rows=[("LaMarcus Aldridge",), ("Marco Belinelli",), ("Danny Green",), ("Aron Baynes",),
               ("Tiago Splitter",), ("Dejounte Murray",)]),
    # OnlyIdTwoSteps (:1172-1188)
    dict(line=1175, query="GO 2 STEPS FROM {P:Tony Parker} OVER like YIELD like._dst",
         rows=[(3394245602834314645,), (-7579316172763586624,), (-7579316172763586624,),
               (5662213458193308137,), (5662213458193308137,)]),
    # ReverselyTwoStep (:1190-1218)
    dict(line=1193, query="GO 2 STEPS FROM hash('Kobe Bryant') OVER like REVERSELY YIELD $$.player.name",
         rows=[("Marc Gasol",), ("Vince Carter",), ("Yao Ming",), ("Grant Hill",)]),
    dict(line=1206, query="GO 2 STEPS FROM hash('Kobe Bryant') OVER * REVERSELY YIELD $$.player.name",
         rows=[("Marc Gasol",), ("Vince Carter",), ("Yao Ming",), ("Grant Hill",)]),
    # Bidirect (:1360-1577)
    dict(line=1363, query="GO FROM {P:Tim Duncan} OVER serve bidirect", rows=[("T:Spurs",)]),
    dict(line=1377, query="GO FROM {P:Tim Duncan} OVER like bidirect",
         rows=[("P:Tony Parker",), ("P:Manu Ginobili",), ("P:Tony Parker",), ("P:Manu Ginobili",),
               ("P:LaMarcus Aldridge",), ("P:Marco Belinelli",), ("P:Danny Green",), ("P:Aron Baynes",),
               ("P:Boris Diaw",), ("P:Tiago Splitter",), ("P:Dejounte Murray",), ("P:Shaquile O'Neal",)]),
    dict(line=1402, query="GO FROM {P:Tim Duncan} OVER serve, like bidirect",
         rows=[("T:Spurs", 0), (0, "P:Tony Parker"), (0, "P:Manu Ginobili"), (0, "P:Tony Parker"),
               (0, "P:Manu Ginobili"), (0, "P:LaMarcus Aldridge"), (0, "P:Marco Belinelli"),
               (0, "P:Danny Green"), (0, "P:Aron Baynes"), (0, "P:Boris Diaw"), (0, "P:Tiago Splitter"),
               (0, "P:Dejounte Murray"), (0, "P:Shaquile O'Neal")]),
    dict(line=1428, query="GO FROM {P:Tim Duncan} OVER * bidirect",
         rows=[("T:Spurs", 0, 0), (0, "P:Tony Parker", 0), (0, "P:Manu Ginobili", 0), (0, "P:Tony Parker", 0),
               (0, "P:Manu Ginobili", 0), (0, "P:LaMarcus Aldridge", 0), (0, "P:Marco Belinelli", 0),
               (0, "P:Danny Green", 0), (0, "P:Aron Baynes", 0), (0, "P:Boris Diaw", 0),
               (0, "P:Tiago Splitter", 0), (0, "P:Dejounte Murray", 0), (0, "P:Shaquile O'Neal", 0),
               (0, 0, "P:Tony Parker"), (0, 0, "P:Manu Ginobili"), (0, 0, "P:LaMarcus Aldridge"),
               (0, 0, "P:Danny Green"), (0, 0, "P:Tony Parker"), (0, 0, "P:Manu Ginobili")]),
    dict(line=1461, query="GO FROM {P:Tim Duncan} OVER serve bidirect YIELD $$.team.name", rows=[("Spurs",)]),
    dict(line=1473, query="GO FROM {P:Tim Duncan} OVER like bidirect YIELD $$.player.name",
         rows=[("Tony Parker",), ("Manu Ginobili",), ("Tony Parker",), ("Manu Ginobili",),
               ("LaMarcus Aldridge",), ("Marco Belinelli",), ("Danny Green",), ("Aron Baynes",),
               ("Boris Diaw",), ("Tiago Splitter",), ("Dejounte Murray",), ("Shaquile O'Neal",)]),
    dict(line=1498, query="GO FROM {P:Tim Duncan} OVER like bidirect WHERE like.likeness > 90 "
                          "YIELD $^.player.name, like._dst, $$.player.name, like.likeness",
         rows=[("Tim Duncan", "P:Tony Parker", "Tony Parker", 95), ("Tim Duncan", "P:Manu Ginobili", "Manu Ginobili", 95),
               ("Tim Duncan", "P:Tony Parker", "Tony Parker", 95),
               ("Tim Duncan", "P:Dejounte Murray", "Dejounte Murray", 99)]),
    dict(line=1515, query="GO FROM {P:Tim Duncan} OVER * bidirect YIELD $^.player.name, serve._dst, "
                          "$$.team.name, like._dst, $$.player.name",
         rows=[("Tim Duncan", "T:Spurs", "Spurs", 0, ""),
               ("Tim Duncan", 0, "", "P:Tony Parker", "Tony Parker"),
               ("Tim Duncan", 0, "", "P:Manu Ginobili", "Manu Ginobili"),
               ("Tim Duncan", 0, "", "P:Tony Parker", "Tony Parker"),
               ("Tim Duncan", 0, "", "P:Manu Ginobili", "Manu Ginobili"),
               ("Tim Duncan", 0, "", "P:LaMarcus Aldridge", "LaMarcus Aldridge"),
               ("Tim Duncan", 0, "", "P:Marco Belinelli", "Marco Belinelli"),
               ("Tim Duncan", 0, "", "P:Danny Green", "Danny Green"),
               ("Tim Duncan", 0, "", "P:Aron Baynes", "Aron Baynes"),
               ("Tim Duncan", 0, "", "P:Boris Diaw", "Boris Diaw"),
               ("Tim Duncan", 0, "", "P:Tiago Splitter", "Tiago Splitter"),
               ("Tim Duncan", 0, "", "P:Dejounte Murray", "Dejounte Murray"),
               ("Tim Duncan", 0, "", "P:Shaquile O'Neal", "Shaquile O'Neal"),
               ("Tim Duncan", 0, "", 0, "Tony Parker"), ("Tim Duncan", 0, "", 0, "Manu Ginobili"),
               ("Tim Duncan", 0, "", 0, "Danny Green"), ("Tim Duncan", 0, "", 0, "LaMarcus Aldridge"),
               ("Tim Duncan", 0, "", 0, "Tony Parker"), ("Tim Duncan", 0, "", 0, "Manu Ginobili")]),
    # FilterPushdown (:1579-...)
    dict(line=1598, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year < 2018",
         pushdown="((serve.start_year>2013)&&(serve.end_year<2018))",
         rows=[("T:Mavericks",), ("T:Kings",), ("T:Bulls",)]),
    dict(line=1614, query="GO FROM {P:Rajon Rondo} OVER serve WHERE !(serve.start_year > 2013 && serve.end_year < 2018)",
         pushdown="!(((serve.start_year>2013)&&(serve.end_year<2018)))",
         rows=[("T:Celtics",), ("T:Pelicans",), ("T:Lakers",)]),
    dict(line=1630, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && $$.team.name == "Kings"',
         pushdown="((serve.start_year>2013)&&true)", rows=[("T:Kings",)]),
    dict(line=1645, query='GO FROM {P:Rajon Rondo} OVER serve WHERE $$.team.name == "Celtics" && $$.team.name == "Kings"',
         pushdown=None, empty=True),
    dict(line=1659, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && '
                          '(serve.end_year < 2018 || $$.team.name == "Kings")',
         pushdown="((serve.start_year>2013)&&true)",
         rows=[("T:Mavericks",), ("T:Kings",), ("T:Bulls",)]),
    dict(line=1676, query='GO FROM {P:Rajon Rondo} OVER serve WHERE (serve.end_year < 2018 || '
                          '$$.team.name == "Kings")&& serve.start_year > 2013',
         pushdown="(true&&(serve.start_year>2013))",
         rows=[("T:Mavericks",), ("T:Kings",), ("T:Bulls",)]),
    # FilterPushdown, rest of the section (:1751-2275; the $-.id pipe case at :2061 is out of scope)
    dict(line=1754, query='GO FROM {P:Rajon Rondo} OVER serve WHERE $$.team.name == "Celtics" || $$.team.name == "Kings"',
         pushdown=None, rows=[("T:Celtics",), ("T:Kings",)]),
    dict(line=1779, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year < 2018 '
                          '&& $$.team.name == "Kings"',
         pushdown="(((serve.start_year>2013)&&(serve.end_year<2018))&&true)", rows=[("T:Kings",)]),
    dict(line=1804, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && $$.team.name == "Kings" '
                          '&& serve.end_year < 2018',
         pushdown="(((serve.start_year>2013)&&true)&&(serve.end_year<2018))", rows=[("T:Kings",)]),
    dict(line=1830, query='GO FROM {P:Rajon Rondo} OVER serve WHERE $$.team.name == "Kings" && serve.start_year > 2013 '
                          '&& serve.end_year < 2018',
         pushdown="((true&&(serve.start_year>2013))&&(serve.end_year<2018))", rows=[("T:Kings",)]),
    dict(line=1857, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year == 2013 "
                          "OR serve.start_year > 2013 && serve.end_year < 2018",
         pushdown="((serve.start_year==2013)||((serve.start_year>2013)&&(serve.end_year<2018)))", rows=list(RK)),
    dict(line=1886, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year <= 2015 "
                          "OR serve.start_year >= 2015 && serve.end_year < 2018",
         pushdown="(((serve.start_year>2013)&&(serve.end_year<=2015))||((serve.start_year>=2015)&&(serve.end_year<2018)))",
         rows=list(RK)),
    dict(line=1916, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year <= 2015 '
                          '&& $$.team.name == "Mavericks" OR serve.start_year >= 2015 && serve.end_year < 2018',
         pushdown="((((serve.start_year>2013)&&(serve.end_year<=2015))&&true)"
                  "||((serve.start_year>=2015)&&(serve.end_year<2018)))", rows=list(RK)),
    dict(line=1946, query='GO FROM {P:Rajon Rondo} OVER serve WHERE $$.team.name == "Pelicans" '
                          'OR serve.start_year > 2013 && serve.end_year < 2018',
         pushdown=None, rows=list(RK) + [("T:Pelicans",)]),
    dict(line=1975, query='GO FROM {P:Rajon Rondo} OVER serve WHERE $$.team.name == "Pelicans" '
                          'OR serve.start_year > 2013 && serve.end_year <= 2015 '
                          'OR serve.start_year >= 2015 && serve.end_year < 2018',
         pushdown=None, rows=list(RK) + [("T:Pelicans",)]),
    dict(line=2006, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year <= 2015 "
                          "XOR serve.start_year >= 2015 && serve.end_year < 2018",
         pushdown="(((serve.start_year>2013)&&(serve.end_year<=2015))XOR((serve.start_year>=2015)&&(serve.end_year<2018)))",
         rows=list(RK)),
    dict(line=2035, query='GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year > 2013 && serve.end_year <= 2015 '
                          '&& $$.team.name == "Mavericks" XOR serve.start_year >= 2015 && serve.end_year < 2018',
         pushdown=None, rows=list(RK)),
    dict(line=2090, query="GO FROM {P:Tim Duncan} OVER serve WHERE serve._src == {P:Tim Duncan} && serve._rank == 0 "
                          "&& serve._dst == {T:Spurs} YIELD serve._dst AS id",
         pushdown="(((serve._src==5662213458193308137)&&(serve._rank==0))&&(serve._dst==7193291116733635180))",
         rows=[("T:Spurs",)]),
    dict(line=2116, query="GO FROM {P:Rajon Rondo} OVER serve WHERE udf_is_in(serve._dst, 1, 2, 3)",
         pushdown="udf_is_in(serve._dst,1,2,3)", empty=True),
    dict(line=2137, query="GO FROM {P:Rajon Rondo} OVER serve WHERE udf_is_in(serve._dst, {T:Celtics}, 2, 3)",
         pushdown="udf_is_in(serve._dst,{T:Celtics},2,3)", rows=[("T:Celtics",)]),
    dict(line=2161, query='GO FROM {P:Rajon Rondo} OVER serve WHERE udf_is_in("test", $$.team.name)',
         pushdown=None, empty=True),
    dict(line=2182, query='GO FROM {P:Tim Duncan} OVER serve WHERE udf_is_in($^.player.name, "Tim Duncan")',
         pushdown="udf_is_in($^.player.name,Tim Duncan)", rows=[("T:Spurs",)]),
    dict(line=2205, query='GO FROM {P:Tim Duncan} OVER serve WHERE !udf_is_in($^.player.name, "Tim Duncan")',
         pushdown="!(udf_is_in($^.player.name,Tim Duncan))", empty=True),
    dict(line=2228, query="GO FROM {P:Boris Diaw} OVER serve WHERE $$.team.name CONTAINS Haw "
                          "YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name",
         pushdown=None, rows=[("Boris Diaw", 2003, 2005, "Hawks")]),
    dict(line=2253, query='GO FROM {P:Boris Diaw} OVER serve WHERE (string)serve.start_year CONTAINS "05" '
                          '&& $^.player.name CONTAINS "Boris" '
                          'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name',
         pushdown="(((string)serve.start_year CONTAINS 05)&&($^.player.name CONTAINS Boris))",
         rows=[("Boris Diaw", 2005, 2008, "Suns")]),
    # DuplicateColumnName (:2279-2297)
    dict(line=2282, query="GO FROM {P:Tim Duncan} OVER serve YIELD serve._dst, serve._dst", rows=[("T:Spurs", "T:Spurs")]),
    # Contains (:2308-2401)
    dict(line=2312, query="GO FROM {P:Boris Diaw} OVER serve WHERE $$.team.name CONTAINS Haw "
                          "YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name",
         rows=[("Boris Diaw", 2003, 2005, "Hawks")]),
    dict(line=2332, query='GO FROM {P:Boris Diaw} OVER serve WHERE (string)serve.start_year CONTAINS "05" '
                          'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name',
         rows=[("Boris Diaw", 2005, 2008, "Suns")]),
    dict(line=2352, query='GO FROM {P:Boris Diaw} OVER serve WHERE $^.player.name CONTAINS "Boris" '
                          'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name',
         rows=[("Boris Diaw", 2003, 2005, "Hawks"), ("Boris Diaw", 2005, 2008, "Suns"),
               ("Boris Diaw", 2008, 2012, "Hornets"), ("Boris Diaw", 2012, 2016, "Spurs"),
               ("Boris Diaw", 2016, 2017, "Jazz")]),
    dict(line=2376, query='GO FROM {P:Boris Diaw} OVER serve WHERE !($^.player.name CONTAINS "Boris") '
                          'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name', empty=True),
    dict(line=2390, query='GO FROM {P:Boris Diaw} OVER serve WHERE "Leo" CONTAINS "Boris" '
                          'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name', empty=True),
    # WithIntermediateData: GO M TO N STEPS (:2403-2841; the two REVERSELY over * blocks at :2808-2841
    # assert nothing and are left out)
    dict(line=2408, query="GO 0 TO 0 STEPS FROM {P:Tony Parker} OVER like YIELD DISTINCT like._dst", empty=True),
    dict(line=2421, query="GO 1 TO 2 STEPS FROM {P:Tony Parker} OVER like YIELD DISTINCT like._dst",
         rows=[("P:Tony Parker",), ("P:Manu Ginobili",), ("P:LaMarcus Aldridge",), ("P:Tim Duncan",)]),
    dict(line=2437, query="GO 0 TO 2 STEPS FROM {P:Tony Parker} OVER like YIELD DISTINCT like._dst",
         rows=[("P:Tony Parker",), ("P:Manu Ginobili",), ("P:LaMarcus Aldridge",), ("P:Tim Duncan",)]),
    dict(line=2454, query="GO 1 TO 2 STEPS FROM {P:Tony Parker} OVER like "
                          "YIELD DISTINCT like._dst, like.likeness, $$.player.name",
         rows=MTON_PROPS),
    dict(line=2474, query="GO 0 TO 2 STEPS FROM {P:Tony Parker} OVER like "
                          "YIELD DISTINCT like._dst, like.likeness, $$.player.name",
         rows=MTON_PROPS),
    dict(line=2494, query="GO 1 TO 3 STEPS FROM {P:Tim Duncan} OVER serve", rows=[("T:Spurs",)]),
    dict(line=2506, query="GO 0 TO 3 STEPS FROM {P:Tim Duncan} OVER serve", rows=[("T:Spurs",)]),
    dict(line=2518, query="GO 2 TO 3 STEPS FROM {P:Tim Duncan} OVER serve", empty=True),
    dict(line=2532, query="GO 1 TO 2 STEPS FROM {P:Tony Parker} OVER like REVERSELY YIELD DISTINCT like._dst",
         rows=MTON_REV),
    dict(line=2556, query="GO 0 TO 2 STEPS FROM {P:Tony Parker} OVER like REVERSELY YIELD DISTINCT like._dst",
         rows=MTON_REV),
    dict(line=2580, query="GO 2 TO 2 STEPS FROM {P:Tony Parker} OVER like REVERSELY YIELD DISTINCT like._dst",
         rows=MTON_REV[1:]),
    dict(line=2603, query="GO 1 TO 3 STEPS FROM {T:Spurs} OVER serve REVERSELY", rows=MTON_SPURS),
    dict(line=2632, query="GO 0 TO 3 STEPS FROM {T:Spurs} OVER serve REVERSELY", rows=MTON_SPURS),
    dict(line=2664, query="GO 1 TO 2 STEPS FROM {P:Tony Parker} OVER like BIDIRECT YIELD DISTINCT like._dst",
         rows=MTON_BI),
    dict(line=2695, query="GO 0 TO 2 STEPS FROM {P:Tony Parker} OVER like BIDIRECT YIELD DISTINCT like._dst",
         rows=MTON_BI),
    dict(line=2727, query="GO 1 TO 2 STEPS FROM {P:Russell Westbrook} OVER * YIELD serve._dst, like._dst",
         rows=MTON_STAR),
    dict(line=2747, query="GO 0 TO 2 STEPS FROM {P:Russell Westbrook} OVER * YIELD serve._dst, like._dst",
         rows=MTON_STAR),
    dict(line=2768, query="GO 1 TO 2 STEPS FROM {P:Russell Westbrook} OVER * "
                          "YIELD serve._dst, like._dst, serve.start_year, like.likeness, $$.player.name",
         rows=MTON_STAR_PROPS),
    dict(line=2789, query="GO 0 TO 2 STEPS FROM {P:Russell Westbrook} OVER * "
                          "YIELD serve._dst, like._dst, serve.start_year, like.likeness, $$.player.name",
         rows=MTON_STAR_PROPS),
    # ErrorMsg (:2844-2854): a team vertex has no player tag -> default ""
    dict(line=2847, query="GO FROM {P:Tim Duncan} OVER serve YIELD $$.player.name as name", rows=[("",)]),
    # ZeroStep (:2856-2883)
    dict(line=2862, query="GO 0 STEPS FROM {P:Tim Duncan} OVER serve BIDIRECT", empty=True),
    dict(line=2874, query="GO 0 STEPS FROM {P:Tim Duncan} OVER serve", empty=True),
    # VertexNotExist (:343-381): no rows at all
    dict(line=357, query="GO FROM hash('NON EXIST VERTEX ID') OVER serve", empty=True),
    dict(line=365, query="GO FROM hash('NON EXIST VERTEX ID') OVER serve YIELD "
                         "$^.player.name, serve.start_year, serve.end_year, $$.team.name", empty=True),
    dict(line=374, query="GO FROM hash('NON EXIST VERTEX ID') OVER serve YIELD DISTINCT "
                         "$^.player.name, serve.start_year, serve.end_year, $$.team.name", empty=True),
    # NonexistentProp (:878-900): E_EXECUTION_ERROR
    dict(line=881, query="GO FROM {P:Tim Duncan} OVER serve YIELD $^.player.test", error=True),
    dict(line=888, query="GO FROM {P:Tim Duncan} OVER serve yield $^.player.test", error=True),
    dict(line=895, query="GO FROM {P:Tim Duncan} OVER serve YIELD serve.test", error=True),
    # is_inCall (:902-923; the two $-.id pipe cases are out of scope)
    dict(line=906, query='GO FROM {P:Boris Diaw} OVER serve WHERE udf_is_in($$.team.name, "Hawks", "Suns") '
                         'YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name',
         rows=[("Boris Diaw", 2003, 2005, "Hawks"), ("Boris Diaw", 2005, 2008, "Suns")]),
    # OneStepOutBound (:97-115)
    dict(line=97, query="GO FROM {P:Rajon Rondo} OVER serve WHERE serve.start_year >= 2013 && serve.end_year <= 2018 "
                        "YIELD $^.player.name, serve.start_year, serve.end_year, $$.team.name",
         rows=[("Rajon Rondo", 2014, 2015, "Mavericks"), ("Rajon Rondo", 2015, 2016, "Kings"),
               ("Rajon Rondo", 2016, 2017, "Bulls"), ("Rajon Rondo", 2017, 2018, "Pelicans")]),
    # MULTI_EDGES, rest (:466-660; the pipe cases at :662-702 are out of scope)
    dict(line=468, query="GO FROM {P:Russell Westbrook} OVER serve, like REVERSELY YIELD serve._src, like._src",
         rows=[(0, "P:Russell Westbrook")] * 3),
    dict(line=482, query="GO FROM {P:Russell Westbrook} OVER serve, like REVERSELY",
         rows=[(0, "P:James Harden"), (0, "P:Dejounte Murray"), (0, "P:Paul George")]),
    dict(line=496, query="GO FROM {P:Russell Westbrook} OVER * REVERSELY YIELD serve._dst, like._dst",
         rows=[(0, "P:James Harden"), (0, "P:Dejounte Murray"), (0, "P:Paul George")]),
    dict(line=510, query="GO FROM {P:Russell Westbrook} OVER * REVERSELY YIELD serve._src, like._src",
         rows=[(0, "P:Russell Westbrook")] * 3),
    dict(line=524, query="GO FROM {P:Russell Westbrook} OVER * REVERSELY",
         rows=[(0, "P:James Harden", 0), (0, "P:Dejounte Murray", 0), (0, "P:Paul George", 0)]),
    dict(line=539, query="GO FROM {P:Manu Ginobili} OVER like, teammate REVERSELY YIELD like.likeness, "
                         "teammate.start_year, $$.player.name",
         rows=[(95, 0, "Tim Duncan"), (95, 0, "Tony Parker"), (90, 0, "Tiago Splitter"), (99, 0, "Dejounte Murray"),
               (0, 2002, "Tim Duncan"), (0, 2002, "Tony Parker")]),
    dict(line=557, query="GO FROM {P:Manu Ginobili} OVER * REVERSELY YIELD like.likeness, teammate.start_year, "
                         "serve.start_year, $$.player.name",
         rows=[(95, 0, 0, "Tim Duncan"), (95, 0, 0, "Tony Parker"), (90, 0, 0, "Tiago Splitter"),
               (99, 0, 0, "Dejounte Murray"), (0, 2002, 0, "Tim Duncan"), (0, 2002, 0, "Tony Parker")]),
    dict(line=575, query="GO FROM {P:Russell Westbrook} OVER serve, like "
                         "YIELD serve.start_year, like.likeness, serve._type, like._type",
         rows=[(2008, 0, 4, 0), (0, 90, 0, 5), (0, 90, 0, 5)]),
    dict(line=591, query="GO FROM {P:Shaquile O'Neal} OVER serve, like",
         rows=[("T:Magic", 0), ("T:Lakers", 0), ("T:Heat", 0), ("T:Suns", 0), ("T:Cavaliers", 0), ("T:Celtics", 0),
               (0, "P:JaVale McGee"), (0, "P:Tim Duncan")]),
    dict(line=611, query="GO FROM {P:Dirk Nowitzki} OVER * YIELD serve._dst, like._dst",
         rows=[("T:Mavericks", 0), (0, "P:Steve Nash"), (0, "P:Jason Kidd"), (0, "P:Dwyane Wade")]),
    dict(line=627, query="GO FROM {P:Paul Gasol} OVER *",
         rows=[("T:Grizzlies", 0, 0), ("T:Lakers", 0, 0), ("T:Bulls", 0, 0), ("T:Spurs", 0, 0), ("T:Bucks", 0, 0),
               (0, "P:Kobe Bryant", 0), (0, "P:Marc Gasol", 0)]),
    dict(line=648, query="GO FROM {P:LaMarcus Aldridge} OVER * YIELD $$.team.name, $$.player.name",
         rows=[("Trail Blazers", ""), ("", "Tim Duncan"), ("", "Tony Parker"), ("Spurs", "")]),
    # NStepQueryHangAndOOM (:3069-3107)
    dict(line=3086, query="GO 1 TO 3 STEPS FROM {P:Tim Duncan} OVER like YIELD like._dst as dst", rows=NSTEP_HANG),
    dict(line=3103, query="GO 1 TO 40 STEPS FROM {P:Tim Duncan} OVER like YIELD like._dst as dst", ok_only=True),
]

# Pipes and variables (GoTest.cpp): `names' is verifyColNames' list when the test checks it.
_SPURS7 = [("T:Spurs",)] * 5 + [("T:Hornets",), ("T:Trail Blazers",)]
_REF_PIPE = [("Tim Duncan", "Manu Ginobili", "Tim Duncan"), ("Tim Duncan", "Tony Parker", "LaMarcus Aldridge"),
             ("Tim Duncan", "Tony Parker", "Manu Ginobili"), ("Tim Duncan", "Tony Parker", "Tim Duncan"),
             ("Chris Paul", "LeBron James", "Ray Allen"), ("Chris Paul", "Carmelo Anthony", "Chris Paul"),
             ("Chris Paul", "Carmelo Anthony", "LeBron James"), ("Chris Paul", "Carmelo Anthony", "Dwyane Wade"),
             ("Chris Paul", "Dwyane Wade", "Chris Paul"), ("Chris Paul", "Dwyane Wade", "LeBron James"),
             ("Chris Paul", "Dwyane Wade", "Carmelo Anthony")]
_REF_PIPE_WHERE = [r for r in _REF_PIPE if r[0] != r[2]]
_REF_PIPE_STAR = [(a, "P:" + b, b, c) for a, b, c in _REF_PIPE]
_REV_LEBRON = ([("Cavaliers", n) for n in ("Kyrie Irving", "Dwyane Wade", "Shaquile O'Neal", "Danny Green",
                                          "LeBron James", "LeBron James")] * 2 +
               [("Heat", n) for n in ("Dwyane Wade", "Dwyane Wade", "LeBron James", "Ray Allen",
                                     "Shaquile O'Neal", "Amar'e Stoudemire")] +
               [("Lakers", n) for n in ("Kobe Bryant", "LeBron James", "Rajon Rondo", "Steve Nash", "Paul Gasol",
                                       "Shaquile O'Neal", "JaVale McGee", "Dwight Howard")])
_MANU_REV = [("T:Spurs",), ("T:Spurs",), ("T:Hornets",), ("T:Spurs",), ("T:Hawks",), ("T:76ers",), ("T:Spurs",)]
_TD = "P:Tim Duncan"
_TD12 = ([(_TD, "P:Tony Parker"), (_TD, "P:Manu Ginobili")] * 2 +
         [(_TD, _TD)] * 4 + [(_TD, "P:Manu Ginobili")] * 2 + [(_TD, "P:LaMarcus Aldridge")] * 2)
_TD12_PROPS = [(_TD, "P:Tony Parker", "P:Tony Parker", 95), (_TD, "P:Tony Parker", "P:Manu Ginobili", 95),
               (_TD, "P:Manu Ginobili", "P:Tony Parker", 95), (_TD, "P:Manu Ginobili", "P:Manu Ginobili", 95),
               (_TD, "P:Tony Parker", _TD, 95), (_TD, "P:Tony Parker", "P:Manu Ginobili", 95),
               (_TD, "P:Tony Parker", "P:LaMarcus Aldridge", 90), (_TD, "P:Tony Parker", _TD, 90),
               (_TD, "P:Manu Ginobili", _TD, 95), (_TD, "P:Manu Ginobili", "P:Manu Ginobili", 95),
               (_TD, "P:Manu Ginobili", "P:LaMarcus Aldridge", 90), (_TD, "P:Manu Ginobili", _TD, 90)]
_DG = [("P:Danny Green", _TD, "P:" + n) for n in ("Tony Parker", "Manu Ginobili", "LaMarcus Aldridge", "Danny Green")]
_TP, _MG, _LA = "P:Tony Parker", "P:Manu Ginobili", "P:LaMarcus Aldridge"
_OVERLAP = [(_TP, x, a, b) for x in (_TD, _MG, _LA)
            for a, b in ((_TD, _MG), (_TD, _TP), (_LA, _TP), (_MG, _TD), (_LA, _TD))]
_TMG = "P:Tracy McGrady"

PIPE_CASES = [
    # OneStepOutBound (:55-69): a constant YIELD sentence feeding GO FROM $-.vid
    dict(line=55, query="YIELD {P:Tim Duncan} as vid | GO FROM $-.vid OVER serve", names=["serve._dst"],
         rows=[("T:Spurs",)]),
    dict(line=118, query="GO FROM {P:Boris Diaw} OVER like YIELD like._dst as id | GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve", names=["serve._dst"], rows=_SPURS7),
    dict(line=176, query="$var = GO FROM {P:Tracy McGrady} OVER like YIELD like._dst as id; "
                         "GO FROM $var.id OVER like", names=["like._dst"], rows=[(_TMG,), (_LA,)]),
    dict(line=198, query="$var = (GO FROM {P:Tracy McGrady} OVER like YIELD like._dst as id | GO FROM $-.id OVER "
                         "like YIELD like._dst as id); GO FROM $var.id OVER like", names=["like._dst"],
         rows=[("P:Kobe Bryant",), ("P:Grant Hill",), ("P:Rudy Gay",), (_TP,), (_TD,)]),
    dict(line=226, query="GO FROM $var OVER like", error=True),
    dict(line=236, query="$var = GO FROM -1 OVER like YIELD like._dst as id; GO FROM $var.id OVER like", empty=True),
    dict(line=304, query="GO FROM {P:Boris Diaw} OVER like YIELD like._dst as id | GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve YIELD DISTINCT serve._dst, $$.team.name",
         names=["serve._dst", "$$.team.name"],
         rows=[("T:Spurs", "Spurs"), ("T:Hornets", "Hornets"), ("T:Trail Blazers", "Trail Blazers")]),
    dict(line=398, query="GO FROM {P:Nobody} OVER serve | GO FROM $-.serve_id OVER serve", empty=True),
    dict(line=405, query="GO FROM {P:Nobody} OVER like YIELD like._dst as id | GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve", empty=True),
    dict(line=414, query="GO FROM {P:Nobody} OVER like YIELD like._dst as id | (GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve)", empty=True),
    dict(line=141, query="GO FROM {P:Boris Diaw} OVER like YIELD like._dst as id | ( GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve )", names=["serve._dst"], rows=_SPURS7),
    dict(line=665, query="GO FROM {P:Boris Diaw} OVER like, serve YIELD like._dst as id | ( GO FROM $-.id OVER "
                         "like YIELD like._dst as id | GO FROM $-.id OVER serve )", rows=_SPURS7),
    dict(line=686, query="GO FROM {P:Boris Diaw} OVER * YIELD like._dst as id | ( GO FROM $-.id OVER like "
                         "YIELD like._dst as id | GO FROM $-.id OVER serve )", rows=_SPURS7),
    dict(line=708, query="GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS name, "
                         "like._dst AS id | GO FROM $-.id OVER like YIELD $-.name, $^.player.name, $$.player.name",
         names=["$-.name", "$^.player.name", "$$.player.name"], rows=_REF_PIPE),
    dict(line=737, query="GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS name, "
                         "like._dst AS id | GO FROM $-.id OVER like WHERE $-.name != $$.player.name "
                         "YIELD $-.name, $^.player.name, $$.player.name",
         names=["$-.name", "$^.player.name", "$$.player.name"], rows=_REF_PIPE_WHERE),
    dict(line=763, query="GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS name, "
                         "like._dst AS id | GO FROM $-.id OVER like YIELD $-.*, $^.player.name, $$.player.name",
         rows=_REF_PIPE_STAR),
    dict(line=795, query="$var = GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS "
                         "name, like._dst AS id; GO FROM $var.id OVER like YIELD $var.name, $^.player.name, "
                         "$$.player.name", names=["$var.name", "$^.player.name", "$$.player.name"], rows=_REF_PIPE),
    dict(line=824, query="$var = GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS "
                         "name, like._dst AS id; GO FROM $var.id OVER like WHERE $var.name != $$.player.name "
                         "YIELD $var.name, $^.player.name, $$.player.name",
         names=["$var.name", "$^.player.name", "$$.player.name"], rows=_REF_PIPE_WHERE),
    dict(line=850, query="$var = GO FROM hash('Tim Duncan'),hash('Chris Paul') OVER like YIELD $^.player.name AS "
                         "name, like._dst AS id; GO FROM $var.id OVER like YIELD $var.*, $^.player.name, "
                         "$$.player.name", rows=_REF_PIPE_STAR),
    dict(line=925, query="GO FROM {P:Tim Duncan} OVER like YIELD like._dst AS id | GO FROM $-.id OVER serve "
                         "WHERE udf_is_in($-.id, {P:Tony Parker}, 123)", names=["serve._dst"],
         rows=[("T:Spurs",), ("T:Hornets",)]),
    dict(line=945, query="GO FROM {P:Tim Duncan} OVER like YIELD like._dst AS id | GO FROM $-.id OVER serve "
                         "WHERE udf_is_in($-.id, {P:Tony Parker}, 123) && 1 == 1", names=["serve._dst"],
         rows=[("T:Spurs",), ("T:Hornets",)]),
    dict(line=1223, query="GO FROM hash('LeBron James') OVER serve YIELD serve._dst AS id | GO FROM $-.id OVER "
                          "serve REVERSELY YIELD $^.team.name, $$.player.name", rows=_REV_LEBRON),
    dict(line=1258, query="GO FROM hash('LeBron James') OVER serve YIELD serve._dst AS id | GO FROM $-.id OVER "
                          "serve REVERSELY WHERE $$.player.name != 'LeBron James' YIELD $^.team.name, "
                          "$$.player.name", rows=[r for r in _REV_LEBRON if r[1] != "LeBron James"]),
    dict(line=1291, query="GO FROM hash('Manu Ginobili') OVER like REVERSELY YIELD like._dst AS id | "
                          "GO FROM $-.id OVER serve", rows=_MANU_REV),
    dict(line=1309, query="GO FROM hash('Manu Ginobili') OVER * REVERSELY YIELD like._dst AS id | "
                          "GO FROM $-.id OVER serve", rows=_MANU_REV),
    dict(line=2063, query="GO FROM {P:Tim Duncan} OVER like YIELD like._dst AS id | GO FROM $-.id OVER serve "
                          "WHERE $^.player.name == \"Tony Parker\" && serve.start_year > 2013",
         names=["serve._dst"], rows=[("T:Hornets",)]),
    dict(line=2297, query="GO FROM {P:Tim Duncan} OVER like YIELD like._dst AS id, like.likeness AS id | "
                          "GO FROM $-.id OVER serve", error=True),
    dict(line=2888, query="GO FROM {P:Tim Duncan} OVER like YIELD like._src as src, like._dst as dst | GO FROM "
                          "$-.src OVER like YIELD $-.src as src, like._dst as dst, $^.player.name, $$.player.name",
         rows=[(_TD, _TP, "Tim Duncan", "Tony Parker"), (_TD, _MG, "Tim Duncan", "Manu Ginobili")] * 2),
    dict(line=2911, query="$a = GO FROM {P:Tim Duncan} OVER like YIELD like._src as src, like._dst as dst; "
                          "GO FROM $a.src OVER like YIELD $a.src as src, like._dst as dst",
         rows=[(_TD, _TP), (_TD, _MG)] * 2),
    dict(line=2930, query="GO FROM {P:Tim Duncan} OVER like YIELD like._src as src, like._dst as dst | GO 1 TO 2 "
                          "STEPS FROM $-.src OVER like YIELD $-.src as src, like._dst as dst", rows=_TD12),
    dict(line=2957, query="GO FROM {P:Tim Duncan} OVER like YIELD like._src as src, like._dst as dst | GO 1 TO 2 "
                          "STEPS FROM $-.src OVER like YIELD $-.src as src, $-.dst, like._dst as dst, like.likeness",
         rows=_TD12_PROPS),
    dict(line=2986, query="GO FROM {P:Danny Green} OVER like YIELD like._src AS src, like._dst AS dst | GO FROM "
                          "$-.dst OVER teammate YIELD $-.src AS src, $-.dst, teammate._dst AS dst", rows=_DG),
    dict(line=3004, query="$a = GO FROM {P:Danny Green} OVER like YIELD like._src AS src, like._dst AS dst; GO FROM "
                          "$a.dst OVER teammate YIELD $a.src AS src, $a.dst, teammate._dst AS dst", rows=_DG),
    dict(line=3047, query="GO FROM {P:Tony Parker} OVER like YIELD like._src as src, like._dst as dst | GO 2 STEPS "
                          "FROM $-.src OVER like YIELD $-.src, $-.dst, like._src, like._dst", rows=_OVERLAP),
    dict(line=3057, query="$a = GO FROM {P:Tony Parker} OVER like YIELD like._src as src, like._dst as dst; GO 2 "
                          "STEPS FROM $a.src OVER like YIELD $a.src, $a.dst, like._src, like._dst", rows=_OVERLAP),
    # NStepQueryHangAndOOM (:3069-3107): the constant YIELD sentence feeding the M TO N walk
    dict(line=3094, query="YIELD {P:Tim Duncan} as id | GO 1 TO 3 STEPS FROM $-.id OVER like YIELD like._dst as dst",
         names=["dst"], rows=NSTEP_HANG),
]
