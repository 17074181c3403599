"""Known answers transcribed from the reference GoTest suite (src/graph/test/GoTest.cpp) on the
NBA fixture (tests/golden/nba.json). Data only: queries and expected rows.

Placeholders: {P:<name>} / {T:<name>} in a query are replaced by the player / team vid
(std::hash<std::string>(name), TraverseTestBase.h:122-126); "P:<name>" / "T:<name>" in an
expected row stand for that vid. Rows are compared sorted, as verifyResult does
(src/graph/test/TestBase.h:188-233). "empty": the response had no rows.
"""

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
]
