"""monitor/cluster"""
