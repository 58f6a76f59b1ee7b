"""monitor/uav"""
