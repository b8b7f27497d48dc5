"""helloworld dataprep examples (JoinsAndAggregates.scala, ConditionalAggregation.scala) on the reference's
own EmailDataset / WebVisitsDataset CSVs, checked against the expected output printed in those files."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples"))


def test_joins_and_aggregates_example():
    import dataprep_joins_aggregates as ex
    rows = ex.main([])
    assert sorted(rows) == ["123", "456", "789"]
    assert rows["123"] == {"ctr": 1.0, "numClicksTomorrow": 1.0, "numClicksYday": 2.0, "numSendsLastWeek": 1.0}
    assert rows["456"]["numClicksTomorrow"] == 1.0
    assert rows["789"]["numSendsLastWeek"] == 1.0
    assert rows["789"]["numClicksTomorrow"] is None and rows["789"]["numClicksYday"] is None


def test_conditional_aggregation_example():
    import dataprep_conditional_aggregation as ex
    rows = ex.main([])
    assert rows == {"xyz@salesforce.com": {"numPurchasesNextDay": 1.0, "numVisitsWeekPrior": 3.0},
                    "lmn@salesforce.com": {"numPurchasesNextDay": 1.0, "numVisitsWeekPrior": 0.0},
                    "abc@salesforce.com": {"numPurchasesNextDay": 0.0, "numVisitsWeekPrior": 1.0}}
