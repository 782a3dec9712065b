"""CPU oracle for the row-update apply path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package.  The product path (parameter_server_amd) never imports it.
"""
