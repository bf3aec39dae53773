"""TEST INFRASTRUCTURE ONLY — CPU oracle for the zipkin-aggregate dependency path.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
Nothing in zipkin_amd/ (the product) imports, links or executes anything under oracle/.
"""
